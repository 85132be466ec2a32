#!/usr/bin/env python3
"""Render a rocprofv3 --stats kernel table (trace_kernel_stats.csv) as markdown.
   python scripts/stats_md.py DIR "title" "command" [bench-json-log ...]"""
import csv
import json
import sys
from pathlib import Path

d, title, cmd = Path(sys.argv[1]), sys.argv[2], sys.argv[3]
print(f"# {title}\n\nCommand: `{cmd}`\n")
print("| kernel | calls | avg ms | % |\n|---|---|---|---|")
for r in csv.DictReader(open(d / "trace_kernel_stats.csv")):
    print(f"| `{r['Name'][:100]}` | {r['Calls']} | {float(r['AverageNs'])/1e6:.3f} | "
          f"{float(r['Percentage']):.2f} |")
for log in sys.argv[4:]:
    for line in open(log):
        if line.startswith("{"):
            j = json.loads(line)
            c = j["config"]
            print(f"\nbench.py ({Path(log).name}): {c['model']}, kernel {c['kernel']}, "
                  f"{j['steps']} steps: **{j['value']:.2f} GDoF/s**, {j['ms_per_step']:.3f} ms/step, "
                  f"y_norm {c['y_norm']:.16g}")
