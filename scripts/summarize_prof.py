#!/usr/bin/env python3
"""Summarise a scripts/prof_fused.sh output directory (kernel stats + PMC)."""
import collections
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
flt = sys.argv[2] if len(sys.argv) > 2 else "lap_fused_kernel"
rows = list(csv.DictReader(open(d / "trace_kernel_stats.csv")))
print("kernel                                                       calls   avg_us    pct")
for r in rows[:10]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} {float(r['Percentage']):6.2f}")
agg = collections.defaultdict(float)
cnt = collections.Counter()
for f in sorted(d.glob("pmc*_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if flt in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[r["Counter_Name"]] += 1
print(f"\nPMC averages per dispatch of kernels matching '{flt}':")
for k in sorted(agg):
    print(f"  {k:28s} {agg[k] / cnt[k]:.4g}")
if "SQ_WAVE_CYCLES" in agg:
    w = agg["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
              "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if k in agg:
            print(f"  {k:28s} {100 * agg[k] / w:5.1f}% of wave cycles")
