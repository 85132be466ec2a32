#!/usr/bin/env python3
"""Summarise a scripts/job_prof3.sh directory: kernel table + PMC per kernel family."""
import collections
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
out = []
rows = list(csv.DictReader(open(d / "trace_kernel_stats.csv")))
out.append("| kernel | calls | avg us | % |")
out.append("|---|---|---|---|")
for r in rows[:12]:
    out.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | "
               f"{float(r['Percentage']):.2f} |")
for fam in ("lap_fused3_kernel", "cg_update_iface_kernel"):
    agg = collections.defaultdict(float)
    cnt = collections.Counter()
    for f in sorted(d.glob("pmc*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if fam in name and (fam != "lap_fused3_kernel" or name.replace(" ", "").count(",1,1>")):
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[r["Counter_Name"]] += 1
    if not agg:
        continue
    out.append(f"\nPMC per dispatch, `{fam}` (CG instance):\n")
    out.append("| counter | value |")
    out.append("|---|---|")
    for k in sorted(agg):
        out.append(f"| {k} | {agg[k] / cnt[k]:.4g} |")
    w = agg.get("SQ_WAVE_CYCLES", 0) / max(cnt.get("SQ_WAVE_CYCLES", 1), 1)
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS"):
            if k in agg:
                out.append(f"| {k} / SQ_WAVE_CYCLES | {100 * agg[k] / cnt[k] / w:.1f} % |")
print("\n".join(out))
