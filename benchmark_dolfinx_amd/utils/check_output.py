"""Golden JSON check of a `bench_dolfinx` output file (the reference's
src/test_output.py:1-19, used by its CI after the 1- and 2-rank runs of
`--ndofs=1000 --degree=3 --qmode=0 --nreps=1 --mat_comp --float=64`).

    python -m benchmark_dolfinx_amd.utils.check_output a.json [b.json ...]
"""

from __future__ import annotations

import json
import sys

import numpy as np

GOLDEN_Y_NORM = 9.912865833415553  # src/test_output.py:19


def check(path: str) -> dict:
    with open(path) as fh:
        data = json.load(fh)
    out = data["output"]
    assert out["ndofs_global"] == 1000, out["ndofs_global"]
    assert np.isclose(out["y_norm"], out["z_norm"]), (out["y_norm"], out["z_norm"])
    assert np.isclose(out["y_norm"], GOLDEN_Y_NORM), out["y_norm"]
    return data


def main(argv=None) -> int:
    for p in (argv if argv is not None else sys.argv[1:]):
        check(p)
        print(f"{p}: ok")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
