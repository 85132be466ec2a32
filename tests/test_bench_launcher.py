"""bench.py's own N-rank launcher (no torchrun): `python bench.py --gpus N`
starts N ranks before anything touches the GPU, relays rank 0's JSON line,
and fails fast (siblings killed, non-zero exit) when a rank fails.  Run here
on the CPU platform (gloo); the GPU path is the same code with RCCL."""

import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    env.update(kw)
    return env


def _bench(args, timeout=300, **env):
    return subprocess.run([sys.executable, "bench.py", "--platform", "cpu", *args], cwd=ROOT,
                          env=_env(**env), capture_output=True, text=True, timeout=timeout)


def _line(r):
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [s for s in r.stdout.strip().splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout  # exactly one JSON record (rank 0's)
    return json.loads(lines[0])


def test_self_launch_four_ranks_matches_one_rank():
    common = ["--steps", "3", "--warmup", "1", "--profile-steps", "0"]
    one = _line(_bench(["--gpus", "1", "--dofs-per-gpu", "24000", *common]))
    four = _line(_bench(["--gpus", "4", "--dofs-per-gpu", "6000", *common]))
    assert one["n_gpus"] == 1 and four["n_gpus"] == 4
    assert four["config"]["comm"]["torch_world"] == 4
    assert four["config"]["comm"]["torch_backend"] == "gloo"
    assert four["config"]["parallelism"].startswith("dd4")
    # same global mesh (weak scaling: 4 x 6000 = 1 x 24000) -> same CG iterate
    assert four["config"]["mesh"] == one["config"]["mesh"]
    y1, y4 = one["config"]["y_norm"], four["config"]["y_norm"]
    assert abs(y1 - y4) <= 1e-12 * abs(y1), (y1, y4)
    c = four["config"]["comm"]
    assert c["rank_ms_per_step_max"] >= c["rank_ms_per_step_min"] > 0


def test_self_launch_kills_siblings_when_a_rank_fails():
    t0 = time.time()
    r = _bench(["--gpus", "3", "--dofs-per-gpu", "5000", "--steps", "2", "--warmup", "1"],
               timeout=240, BDX_BENCH_FAIL_RANK="2")
    assert r.returncode != 0
    assert "stopping the other ranks" in r.stderr
    assert not [s for s in r.stdout.splitlines() if s.startswith("{")]
    # ranks 0/1 would wait for rank 2 in the rendezvous forever; the launcher
    # must end them well before torch's own 600 s timeout
    assert time.time() - t0 < 200


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, "bench.py", "--platform", "cpu", "--gpus", "4"],
                       cwd=ROOT, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
