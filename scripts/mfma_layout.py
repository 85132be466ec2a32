#!/usr/bin/env python3
"""Infer the lane maps of the FP64 MFMA shapes from the probe's dump
(csrc/micro/mfma_f64_shapes.hip, lines "L16 ..." / "L4 ...").

Each operand's lane index (6 bits) is split into three 2-bit fields (for
4x4x4_4b: block, row-or-col, k) in some order; for 16x16x4 the documented map
(A[l&15][l>>4], B[l>>4][l&15], D row (l>>4)+4r, col l&15) is checked.  Prints
the field orders that reproduce D exactly for every trial.

  python scripts/mfma_layout.py gpurun_out/r6_mfma_shapes.txt
"""

from __future__ import annotations

import itertools
import sys

import numpy as np


def parse(path):
    out = {"L16": [], "L4": []}
    for line in open(path):
        tok = line.split()
        if not tok or tok[0] not in out:
            continue
        i = tok.index("A")
        j = tok.index("B")
        k = tok.index("D")
        out[tok[0]].append((np.array(tok[i + 1:j], float), np.array(tok[j + 1:k], float),
                            np.array(tok[k + 1:], float)))
    return out


def check16(trials):
    ok = True
    for a, b, d in trials:
        A = np.zeros((16, 4))
        B = np.zeros((4, 16))
        for lane in range(64):
            A[lane & 15, lane >> 4] = a[lane]
            B[lane >> 4, lane & 15] = b[lane]
        C = A @ B
        for lane in range(64):
            for r in range(4):
                ok &= d[lane * 4 + r] == C[(lane >> 4) + 4 * r, lane & 15]
    return ok


def fields(lane, order):
    """lane bits (0-1, 2-3, 4-5) -> the named fields in `order`."""
    v = [(lane >> (2 * p)) & 3 for p in range(3)]
    return dict(zip(order, v))


def search4(trials):
    names_a = ("blk", "row", "k")
    names_b = ("blk", "col", "k")
    names_d = ("blk", "row", "col")
    hits = []
    for oa in itertools.permutations(names_a):
        for ob in itertools.permutations(names_b):
            for od in itertools.permutations(names_d):
                good = True
                for a, b, d in trials:
                    A = np.zeros((4, 4, 4))
                    B = np.zeros((4, 4, 4))
                    for lane in range(64):
                        f = fields(lane, oa)
                        A[f["blk"], f["row"], f["k"]] = a[lane]
                        g = fields(lane, ob)
                        B[g["blk"], g["k"], g["col"]] = b[lane]
                    C = np.einsum("bik,bkj->bij", A, B)
                    for lane in range(64):
                        h = fields(lane, od)
                        if d[lane] != C[h["blk"], h["row"], h["col"]]:
                            good = False
                            break
                    if not good:
                        break
                if good:
                    hits.append((oa, ob, od))
    return hits


def main(argv=None):
    path = (argv or sys.argv[1:])[0]
    t = parse(path)
    print("16x16x4 documented map:", "OK" if t["L16"] and check16(t["L16"]) else "MISMATCH")
    hits = search4(t["L4"])
    print("4x4x4_4b maps (lane bit pairs 0-1, 2-3, 4-5 carry these fields):")
    for h in hits:
        print("  A", h[0], " B", h[1], " D", h[2])
    if not hits:
        print("  none of the 216 field orders reproduces D")


if __name__ == "__main__":
    main()
