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
    # the metric's Q6 half rides along (own steps / ms_per_step), FP64 and
    # FP32, partition-invariant like the headline
    for rec in (one, four):
        for c in ("q6", "q6f32"):
            comp = rec["companions"][c]
            assert comp.get("error") is None, comp
            assert comp["steps"] == 3 and comp["warmup"] == 1 and comp["degree"] == 6
            assert comp["dtype"] == ("fp64" if c == "q6" else "fp32")
            assert rec[f"{c}_gdofs"] == comp["value"] > 0
        # the north star's random coefficients, on the headline's own clock
        rk = rec["companions"]["random_kappa"]
        assert rk.get("error") is None and rk["kappa"] == "random" and rk["steps"] == 3
        assert rk["degree"] == 3 and rk["mesh"] == rec["config"]["mesh"]
        assert rec["random_kappa_gdofs"] == rk["value"] > 0
    for c, tol in (("q6", 1e-12), ("q6f32", 1e-4), ("random_kappa", 1e-12)):
        a, b = one["companions"][c]["y_norm"], four["companions"][c]["y_norm"]
        assert abs(a - b) <= tol * abs(a), (c, a, b)
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


def test_self_launch_eight_ranks_yz_partition():
    """The 8-GPU driver run's shape on the CPU: 8 self-launched ranks, x kept
    whole (1 x 2 x 4, the GPU partition policy), same CG iterate as 1 rank."""
    common = ["--steps", "2", "--warmup", "1", "--profile-steps", "0", "--companions", "off"]
    one = _line(_bench(["--gpus", "1", "--dofs-per-gpu", "24000", *common]))
    eight = _line(_bench(["--gpus", "8", "--dofs-per-gpu", "3000", *common], timeout=400,
                         BDX_PARTITION="yz"))
    assert eight["n_gpus"] == 8
    # x whole, y and z both split (1x2x4 on the GPU's meshes; 1x4x2 here)
    assert eight["config"]["parallelism"].split()[1] in ("(1x2x4", "(1x4x2")
    assert eight["config"]["comm"]["torch_world"] == 8
    assert eight["config"]["mesh"] == one["config"]["mesh"]
    y1, y8 = one["config"]["y_norm"], eight["config"]["y_norm"]
    assert abs(y1 - y8) <= 1e-12 * abs(y1), (y1, y8)
    assert eight["q6_gdofs"] is None and not eight["companions"]


def test_self_launch_kills_siblings_when_a_rank_fails():
    t0 = time.time()
    r = _bench(["--gpus", "3", "--dofs-per-gpu", "5000", "--steps", "2", "--warmup", "1"],
               timeout=240, BDX_BENCH_FAIL_RANK="2")
    assert r.returncode != 0
    assert "stopping the other ranks" in r.stderr
    # one JSON line, from the launcher: no value, the error
    lines = [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["value"] is None and "exited with" in rec["error"]
    # ranks 0/1 would wait for rank 2 in the rendezvous forever; the launcher
    # must end them well before torch's own 600 s timeout
    assert time.time() - t0 < 200


def test_failed_companion_on_several_ranks_reports_headline_and_error():
    """A secondary measurement that fails on a multi-rank run is fatal (a rank
    that skipped ahead would pair up the wrong collectives), but rank 0 still
    prints one JSON line: the headline it measured and the error."""
    r = _bench(["--gpus", "2", "--dofs-per-gpu", "6000", "--steps", "2", "--warmup", "1",
                "--profile-steps", "0"], timeout=300, BDX_BENCH_FAIL_MEASURE="q6f32")
    assert r.returncode != 0
    lines = [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert "injected failure in the q6f32" in rec["error"]
    assert rec["value"] > 0 and rec["n_gpus"] == 2          # the headline survived
    assert rec["q6_gdofs"] > 0 and rec["q6f32_gdofs"] is None


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, "bench.py", "--platform", "cpu", "--gpus", "4"],
                       cwd=ROOT, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


def test_multirank_run_records_the_reference_data_model():
    """N > 1: after the headline and companions, rank 0's
    record carries the reference data model (dofmap + stored G) on the same
    weak-scaled mesh, timed with the headline's steps / warm-up, and the
    cross-family consistency pair q3~dofmap; here on 2 / 4 / 8 gloo ranks
    with the C++ CPU dofmap operator (the GPU path is the same code with the
    HIP kernel and RCCL, tests/test_gpu_distributed_emulated.py)."""
    one = _line(_bench(["--gpus", "1", "--dofs-per-gpu", "24000", "--steps", "3", "--warmup",
                        "1", "--profile-steps", "0", "--companions", "off"]))
    assert not one["variants"]  # one CPU rank: no variants (GPU-only extras)
    for n in (2, 4, 8):
        rec = _line(_bench(["--gpus", str(n), "--dofs-per-gpu", str(24000 // n), "--steps", "3",
                            "--warmup", "1", "--profile-steps", "0", "--companions", "off"],
                           timeout=400, BDX_PARTITION="yz"))
        dm = rec["variants"]["dofmap"]
        assert dm.get("error") is None, dm
        assert dm["kernel"] == "dofmap" and dm["geometry"] == "dofmap-stored"
        assert dm["steps"] == 3 and dm["warmup"] == 1 and dm["value"] > 0
        assert rec["dofmap_gdofs"] == dm["value"]
        assert dm["mesh"] == rec["config"]["mesh"] == one["config"]["mesh"]
        assert dm["comm"]["torch_world"] == n
        pair = rec["consistency"]["pairs"]["q3~dofmap"]
        assert pair["ok"] and pair["action_norm"] < 1e-12 and pair["y_norm"] < 1e-10, pair
        assert abs(dm["y_norm"] - one["config"]["y_norm"]) <= 1e-10 * one["config"]["y_norm"]
