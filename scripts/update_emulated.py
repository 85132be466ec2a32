#!/usr/bin/env python3
"""Fold emulate_rank.py records (one JSON line per run, "mode": "emulated")
into benchmark_dolfinx_amd/data/emulated_predictions.json, the table bench.py
reads for config.emulated_ms_per_step at N > 1.

  python scripts/update_emulated.py SOURCE_NOTE run1.log [run2.log ...]
"""

from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "benchmark_dolfinx_amd", "data", "emulated_predictions.json")


def main(argv):
    note, paths = argv[0], argv[1:]
    tab = json.load(open(TABLE))
    for p in paths:
        for line in open(p):
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            if d.get("mode") != "emulated" or d["link"]["BDX_EMU_LINK_GBPS"] != 50.0:
                continue
            tab["runs"].setdefault(d["config"], {}).setdefault(d["kernel"], {})[
                str(d["nranks"])] = round(d["ms_per_step"], 4)
            tab["source"][d["kernel"]] = note
    with open(TABLE, "w") as f:
        json.dump(tab, f, indent=1)
    print(json.dumps(tab["runs"]))


if __name__ == "__main__":
    main(sys.argv[1:])
