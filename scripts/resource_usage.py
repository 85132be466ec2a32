#!/usr/bin/env python3
"""Per-kernel VGPR / spill / LDS / occupancy of one HIP TU for gfx950.

usage: python scripts/resource_usage.py benchmark_dolfinx_amd/csrc/hip/<tu>.hip [-- extra hipcc flags]
"""
import re
import subprocess
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from benchmark_dolfinx_amd.ops.build import HIPCC, hip_flags


def main():
    src = sys.argv[1]
    extra = sys.argv[3:] if len(sys.argv) > 2 and sys.argv[2] == "--" else []
    cmd = [HIPCC, *hip_flags(), *extra, "-c", src, "-o", "/tmp/ru.o",
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            name = t.split(":", 1)[1].strip()
            name = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
            cur = {"name": name}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    for r in rows:
        print("%4s vgpr %3s agpr spill %4s lds %6s occ %s  %s" % (
            r.get("VGPRs", "?"), r.get("AGPRs", "0"), r.get("VGPRs Spill", "?"),
            r.get("LDS Size [bytes/block]", "?"), r.get("Occupancy [waves/SIMD]", "?"),
            r["name"][:140]))


if __name__ == "__main__":
    main()
