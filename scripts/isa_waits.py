#!/usr/bin/env python3
"""Summarise the s_waitcnt vmcnt / barrier structure of every kernel in a
device .s file (hipcc --cuda-device-only -S):  python scripts/isa_waits.py f.s"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for m in re.finditer(r'^(_Z\w+):[^\n]*\n', s, re.M):
    name = m.group(1)
    end = s.find('.Lfunc_end', m.end())
    k = s[m.end():end]
    waits = Counter(re.findall(r's_waitcnt[^\n]*vmcnt\((\d+)\)', k))
    print(f"{name[:70]:70s} lines {k.count(chr(10)):5d} barriers {k.count('s_barrier'):3d} "
          f"vmcnt {sorted(waits.items(), key=lambda t: int(t[0]))}")
