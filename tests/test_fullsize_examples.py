"""The committed full-size single-MI355X runs (examples/mi355x/*.json, written by
the CLI through scripts/job_fullsize.sh) against the Kronecker closed form.

The reference publishes its headline JSONs for 64 GPUs (examples/Q3-300M.json,
examples/Q6-500M.json); these are the same configurations at one GPU's share
(300 M / 500 M DoFs).  On the unperturbed box ||u|| and the action-mode ||y||
have an O(n) closed form (oracle.kron_norms), so the GPU results at full size
are pinned to rounding.  The CG-mode y_norm (the iterate after 1000 CG steps)
has no closed form; only u_norm, sizes and the reported rate are checked there.
"""

import json
import os

import pytest

from oracle import kron_norms

EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples",
                  "mi355x")

CASES = [
    # file, mesh, degree, ndofs, float bits, cg
    ("Q3-300M-action.json", (222, 223, 223), 3, 299416300, 64, False),
    ("Q3-300M.json", (222, 223, 223), 3, 299416300, 64, True),
    ("Q6-500M-action.json", (132, 132, 132), 6, 498677257, 64, False),
    ("Q6-500M.json", (132, 132, 132), 6, 498677257, 64, True),
    ("Q6-500M-fp32.json", (132, 132, 132), 6, 498677257, 32, True),
]


@pytest.mark.parametrize("name,mesh,degree,ndofs,bits,cg", CASES)
def test_fullsize_json_matches_closed_form(name, mesh, degree, ndofs, bits, cg):
    d = json.load(open(os.path.join(EX, name)))
    i, o = d["input"], d["output"]
    assert i["p"] == degree and i["qmode"] == 1 and i["scalar_size"] == bits and i["cg"] == cg
    assert o["ndofs_global"] == ndofs and tuple(d["mi355x"]["mesh"]) == mesh
    assert o["ndofs_global"] == (degree * mesh[0] + 1) * (degree * mesh[1] + 1) * (degree * mesh[2] + 1)
    u, y = kron_norms(mesh, degree, 1, False)
    tol = 1e-13 if bits == 64 else 1e-6
    assert abs(o["u_norm"] - u) <= tol * u
    if not cg:
        assert abs(o["y_norm"] - y) <= tol * y
    # the rate is the figure of merit: ndofs * nreps / (1e9 t)
    rate = o["ndofs_global"] * i["nreps"] / (1e9 * o["mat_free_time"])
    assert abs(rate - o["gdof_per_second"]) <= 1e-9 * rate
