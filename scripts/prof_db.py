#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 rocpd database (ROCm 7 default output):
calls, total / mean ms, share, sorted by total time.

usage: python scripts/prof_db.py gpurun_out/.../run_results.db [--top N] [--md]
"""
import sqlite3
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 25
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start) from kernels "
                     f"group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    md = "--md" in sys.argv
    if md:
        print("| kernel | calls | total ms | mean ms | share |\n|---|---|---|---|---|")
    for n, cnt, t in rows[:top]:
        n = n if len(n) < 110 else n[:107] + "..."
        if md:
            print(f"| `{n}` | {cnt} | {t / 1e6:.3f} | {t / 1e6 / cnt:.4f} | {100 * t / tot:.1f} % |")
        else:
            print(f"{cnt:6d} {t / 1e6:10.3f} ms {t / 1e6 / cnt:9.4f} ms {100 * t / tot:5.1f}%  {n}")


if __name__ == "__main__":
    main()
