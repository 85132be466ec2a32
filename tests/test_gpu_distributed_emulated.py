"""Multi-rank GPU code paths on ONE GPU: R ranks run as threads (ThreadComm)
with RCCL semantics emulated (collectives reject host tensors), through the
real bench.py `run()` and the CLI driver.  This is the rehearsal of the
driver's torchrun N = 2/4/8 launches that cannot run on a 1-GPU box."""

import os
import sys

import pytest
import torch

from benchmark_dolfinx_amd.parallel.comm import run_threaded

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _bench(comm, config, total, kernel="auto", geometry="auto"):
    import bench
    a = bench.parse_args(["--config", config, "--dofs-per-gpu", str(total // comm.size),
                          "--steps", "6", "--warmup", "2", "--kernel", kernel,
                          "--geometry", geometry, "--gpus", str(comm.size)])
    out = bench.run(comm, a)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("config,total", [("q3", 2_000_000), ("q6", 3_000_000),
                                          ("q6f32", 3_000_000)])
@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_bench_run_multirank_matches_single(config, total, ranks):
    ref = run_threaded(1, _bench, config, total, emulate="nccl")[0]
    got = run_threaded(ranks, _bench, config, total, emulate="nccl")[0]
    assert got["n_gpus"] == ranks and got["value"] > 0
    assert got["config"]["mesh"] == ref["config"]["mesh"]
    bs = got["config"]["box_stream"]  # the untimed box probe, reduced over ranks
    assert bs["n"] > 0 and 0 < bs["tbps_min"] <= bs["tbps_max"]
    assert 0 < bs["dgemm_tflops_min"] <= bs["dgemm_tflops_max"]
    tol = 1e-11 if config != "q6f32" else 2e-5
    assert abs(got["config"]["y_norm"] - ref["config"]["y_norm"]) <= tol * ref["config"]["y_norm"]
    if config == "q3":
        # N > 1: the reference data model on the same mesh, in-process after
        # the companions, with its per-rank split-schedule timeline and the
        # cross-family consistency pair
        dm = got["variants"]["dofmap"]
        assert dm.get("error") is None, dm
        assert dm["kernel"] == "dofmap" and dm["steps"] == 6 and dm["value"] > 0
        assert got["dofmap_gdofs"] == dm["value"]
        ppr = dm["phases_per_rank"]
        assert ppr is not None and len(ppr) == ranks
        assert all(p["iteration"] > 0 and p["interior_done"] > 0 for p in ppr)
        pair = got["consistency"]["pairs"]["q3~dofmap"]
        assert pair["ok"] and pair["action_norm"] < 1e-12, pair
        assert got["consistency"]["ok"]


@pytest.mark.parametrize("geometry", ["otf-general", "stored"])
def test_bench_run_multirank_other_paths(geometry):
    ref = run_threaded(1, _bench, "q3", 1_000_000, "auto", geometry, emulate="nccl")[0]
    got = run_threaded(4, _bench, "q3", 1_000_000, "auto", geometry, emulate="nccl")[0]
    assert abs(got["config"]["y_norm"] - ref["config"]["y_norm"]) <= 1e-11 * ref["config"]["y_norm"]


def _cli(comm, cg, mat_comp, nreps):
    from benchmark_dolfinx_amd import cli
    from benchmark_dolfinx_amd.fem.mesh import compute_mesh_size
    args, _ = cli.parse_args(["--platform=gpu", "--ndofs_global=60000", "--degree=3",
                              f"--nreps={nreps}", "--geom_perturb_fact=0.1"]
                             + (["--cg"] if cg else []) + (["--mat_comp"] if mat_comp else []))
    nx = compute_mesh_size(60000, 3)
    out, extra = cli.run_benchmark(comm, nx, args, "gpu")
    from benchmark_dolfinx_amd.utils.timing import list_timings
    list_timings(comm)
    torch.cuda.synchronize()
    return out, extra


@pytest.mark.parametrize("cg", [False, True])
def test_cli_driver_multirank_mat_comp(cg):
    ref = run_threaded(1, _cli, cg, True, 5, emulate="nccl")[0]
    got = run_threaded(4, _cli, cg, True, 5, emulate="nccl")[0]
    o, e = got
    assert e["e_norm"] <= 1e-11 * o["z_norm"]
    assert abs(o["y_norm"] - ref[0]["y_norm"]) <= 1e-11 * ref[0]["y_norm"]
