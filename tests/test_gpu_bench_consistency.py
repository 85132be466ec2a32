"""bench.py's cross-family consistency gate.

The headline (fused5) and the reference-data-model variant (dofmap, stored
G) solve the same problem; bench.py compares one operator action of each on
the RHS (||A b|| and a positively weighted sum of (A b)^2) and exits non-zero
when they disagree by more than 1e-9.  Here a 0.1 % error in one entry of the
dofmap kernels' interpolation table (BDX_TEST_CORRUPT_DOFMAP) must fail the
run, and the clean run must pass with gaps at rounding level."""

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(**env):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        e.pop(k, None)
    e.update(env)
    args = [sys.executable, "bench.py", "--dofs-per-gpu", "2000000", "--steps", "3", "--warmup",
            "1", "--companions", "off", "--extras", "on", "--box-probe", "off",
            "--profile-steps", "0"]
    return subprocess.run(args, cwd=ROOT, env=e, capture_output=True, text=True, timeout=420)


def _line(r):
    lines = [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:] + r.stderr[-2000:]
    return json.loads(lines[0])


def test_consistency_gate_passes_and_catches_a_corrupt_dofmap_table():
    ok = _bench()
    assert ok.returncode == 0, ok.stderr[-3000:]
    rec = _line(ok)
    pair = rec["consistency"]["pairs"]["q3~dofmap"]
    assert pair["ok"] and pair["action_norm"] < 1e-12 and pair["action_wdot"] < 1e-12, pair
    assert rec["consistency"]["pairs"]["general~general_trilinear"]["ok"]
    # the MFMA kernel of the data model is timed as its own variant and
    # pinned to the VALU one on the same problem
    var = rec["variants"]
    assert var["dofmap"]["dofmap_core"] == "valu" and var["dofmap_mfma"]["dofmap_core"] == "mfma"
    assert rec["dofmap_mfma_gdofs"] > 0 and rec["q6_dofmap_mfma_gdofs"] > 0
    for key in ("dofmap~dofmap_mfma", "q6_dofmap~q6_dofmap_mfma"):
        pair = rec["consistency"]["pairs"][key]
        assert pair["ok"] and pair["action_norm"] < 1e-12 and pair["action_wdot"] < 1e-12, pair
    bad = _bench(BDX_TEST_CORRUPT_DOFMAP="1")
    assert bad.returncode == 4, (bad.returncode, bad.stderr[-3000:])
    rec = _line(bad)  # the JSON line is still printed
    pair = rec["consistency"]["pairs"]["q3~dofmap"]
    assert not pair["ok"] and not rec["consistency"]["ok"]
    assert pair["action_norm"] > 1e-6
    assert "disagree" in bad.stderr
