#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 counter_collection.csv files (one row per
dispatch x counter); prints kernel, calls, and each counter's per-dispatch mean."""
import collections
import csv
import sys


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.defaultdict(set)
    for p in paths:
        for row in csv.DictReader(open(p)):
            k = row["Kernel_Name"][:70]
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            calls[k].add((p, row["Dispatch_Id"]))
    for k, d in sorted(acc.items(), key=lambda kv: -max(kv[1].values())):
        n = len(calls[k]) or 1
        print(f"{k}  (dispatches {n})")
        for c, v in sorted(d.items()):
            print(f"    {c:28s} {v / n:16.4g}")


if __name__ == "__main__":
    main(sys.argv[1:])
