"""GPU tests of the native CG runtime (csrc/hip/runtime.hip): the overlapped
two-stream schedule (halo exchange hidden under interior tiles) against one
rank, the all-or-nothing construction across ranks, per-operator device
tables under graph replay, re-binding the iterate, hipEvent phase timers,
and bench.py's own entry point on one GPU."""

import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from benchmark_dolfinx_amd.models.fused import FusedLaplacianGPU, fused_supported
from benchmark_dolfinx_amd.models.poisson import MatFreeLaplacianCPU, PoissonProblem
from benchmark_dolfinx_amd.parallel.comm import Comm, run_threaded
from benchmark_dolfinx_amd.solvers.cg import DeviceCG, cg_solve
from benchmark_dolfinx_amd.solvers.native import NativeCGRuntime

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _job(comm, nc, P, nreps, version, partition, pert=0.0, dtype=torch.float64,
         coefficient="constant"):
    pb = PoissonProblem(comm, nc, P, 1, False, dtype, "gpu", pert, coefficient,
                        partition=partition)
    if not fused_supported(pb, version):
        return None
    u = pb.assemble_rhs()
    x = pb.new_vector()
    op = FusedLaplacianGPU(pb, "otf", version, affine=version == 5 or pert == 0.0)
    cg = DeviceCG(pb)
    cg.solve(op, x, u, nreps)
    cg.wait()
    rt = op._rt
    info = (rt.overlap, rt.transport, rt.comm_ranks(), op.runtime) if rt else (
        False, "python", None, op.runtime)
    xn = pb.norm(x)
    op.close()
    return xn, pb.lat.pgrid, info + (tuple(pb.lat.gh),)


# meshes large enough that interior (ghost-free) tiles exist on every rank
@pytest.mark.parametrize("version,P,nc", [(2, 3, (5, 22, 26)), (3, 3, (5, 22, 26)),
                                          (5, 3, (5, 22, 26)), (5, 6, (3, 9, 10)),
                                          (5, 4, (4, 14, 13))])
@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_overlap_schedule_matches_one_rank(ranks, version, P, nc):
    ref = run_threaded(1, _job, nc, P, 12, version, "yz")[0]
    if ref is None:
        pytest.skip(f"fused{version} does not cover P={P}")
    got = run_threaded(ranks, _job, nc, P, 12, version, "yz")
    for xn, pgrid, (overlap, transport, nr, runtime, gh) in got:
        assert pgrid[0] == 1 and runtime == "native" and transport == "thread" and nr == ranks
        # x whole: every rank with an upper (y or z) neighbour splits its tiles
        assert overlap == bool(gh[1] or gh[2]), (overlap, gh)
        assert abs(xn - ref[0]) <= 1e-11 * abs(ref[0]), (xn, ref[0])
    assert any(r[2][0] for r in got)
    # the serial schedule (x split by the min-cut partition) gives the same iterate
    ser = run_threaded(ranks, _job, nc, P, 12, version, "xyz")
    for xn, pgrid, (overlap, *_rest, gh) in ser:
        assert overlap == (pgrid[0] == 1 and bool(gh[1] or gh[2]))
        assert abs(xn - ref[0]) <= 1e-11 * abs(ref[0])


def test_overlap_schedule_random_kappa_fp32():
    nc = (4, 18, 20)
    ref = run_threaded(1, _job, nc, 3, 10, 3, "yz", 0.0, torch.float32, "random")[0]
    got = run_threaded(4, _job, nc, 3, 10, 3, "yz", 0.0, torch.float32, "random")
    assert any(r[2][0] for r in got)
    for xn, _, _info in got:
        assert abs(xn - ref[0]) <= 2e-5 * abs(ref[0])


def test_create_failure_on_one_rank_falls_back_on_every_rank():
    nc = (4, 10, 12)
    ref = run_threaded(1, _job, nc, 3, 8, 2, "yz")[0]
    NativeCGRuntime._inject_fail_rank = 1
    try:
        got = run_threaded(3, _job, nc, 3, 8, 2, "yz")
    finally:
        NativeCGRuntime._inject_fail_rank = None
    for xn, _, (_ov, transport, _nr, runtime, _gh) in got:
        assert runtime == "python" and transport == "python"  # all ranks, not only rank 1
        assert abs(xn - ref[0]) <= 1e-11 * abs(ref[0])


def _host_cg(nc, P, qm, g, n):
    cpu = PoissonProblem(Comm(), nc, P, qm, g, torch.float64, "cpu")
    xc = cpu.new_vector()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), n)
    return cpu, xc


@pytest.mark.parametrize("graph", ["1", "0"])
def test_fused5_operators_keep_their_own_tables_under_graph_replay(monkeypatch, graph):
    """Two fused5 operators of the same (P, T) with different tables (qmode 1
    vs qmode 0 GLL; Gauss) interleave their graph-replayed (BDX_GRAPH=1) or
    eager (0, the default) iterations; each must match its own host CG (a
    shared device table would mix them)."""
    monkeypatch.setenv("BDX_GRAPH", graph)
    nc, P = (3, 4, 5), 5
    cases = [(1, False), (0, False), (1, True)]
    runs = []
    for qm, g in cases:
        pb = PoissonProblem(Comm(), nc, P, qm, g, torch.float64, "gpu")
        if not fused_supported(pb, 5):
            pytest.skip("no fused5 instance")
        op = FusedLaplacianGPU(pb, "otf", 5)
        cg = DeviceCG(pb)
        x = pb.new_vector()
        cg.start(op, x, pb.assemble_rhs())
        runs.append((pb, op, cg, x))
    for _ in range(6):  # interleave: 6 rounds x 4 iterations each, graphs replayed
        for pb, op, cg, x in runs:
            cg.iterate(4)
    torch.cuda.synchronize()
    for (qm, g), (pb, op, cg, x) in zip(cases, runs):
        assert op._rt is not None and op._rt.graphs == (graph == "1")
        cpu, xc = _host_cg(nc, P, qm, g, 24)
        rel = (cpu.owned(x.cpu()) - cpu.owned(xc)).abs().max().item() / xc.abs().max().item()
        assert rel < 1e-10, (qm, g, rel)
        op.close()


@pytest.mark.parametrize("tiled", ["1", "0"])
@pytest.mark.parametrize("graph", ["0", "1"])
@pytest.mark.parametrize("xpair", ["1", "0", "1-nostagger"])
def test_fused5_paired_x_update_any_call_split(monkeypatch, xpair, graph, tiled):
    """fused5's paired lagged x update (kXSave / kXPair in runtime.hip: x is
    read and written every other iteration; on tiled storage staggered, the
    odd tiles pairing on the even tiles' save iterations) against the host
    CG, for call splits that leave 1 or 2 terms pending at the flush that
    ends each call, through iterate, iterate_timed and the profiled
    iterations."""
    monkeypatch.setenv("BDX_XPAIR", xpair[0])
    monkeypatch.setenv("BDX_XSTAGGER", "0" if xpair.endswith("nostagger") else "1")
    monkeypatch.setenv("BDX_GRAPH", graph)
    monkeypatch.setenv("BDX_TILED", tiled)
    nc, P = (4, 5, 6), 3
    pb = PoissonProblem(Comm(), nc, P, 1, False, torch.float64, "gpu")
    if not fused_supported(pb, 5):
        pytest.skip("no fused5 instance")
    op = FusedLaplacianGPU(pb, "otf", 5)
    cg = DeviceCG(pb)
    x = pb.new_vector()
    cg.start(op, x, pb.assemble_rhs())
    assert op._rt is not None and op._rt.tiled == (tiled == "1")
    total = 0
    for kind, n in (("it", 1), ("it", 2), ("it", 5), ("timed", 4), ("prof", 3), ("it", 6),
                    ("timed", 3)):
        if kind == "it":
            cg.iterate(n)
        elif kind == "timed":
            assert len(cg.iterate_timed(n)) == n
        else:
            op._rt.profile(n)
        total += n
        cg.wait()
        cpu, xc = _host_cg(nc, P, 1, False, total)
        rel = (cpu.owned(x.cpu()) - cpu.owned(xc)).abs().max().item() / xc.abs().max().item()
        assert rel < 1e-10, (kind, n, total, rel)
    assert cg.it == total
    op.close()


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_fused5_staggered_pairing_multi_rank(monkeypatch, dtype):
    """Staggered paired x update on 4 threaded ranks (tiled storage, graphs
    off and on) against one x term per iteration: the same iterate."""
    nc, P = (5, 9, 10), 3
    res = {}
    for mode in ("stagger", "single"):
        monkeypatch.setenv("BDX_XPAIR", "1" if mode == "stagger" else "0")
        monkeypatch.setenv("BDX_XSTAGGER", "1")
        monkeypatch.setenv("BDX_TILED", "1")
        res[mode] = run_threaded(4, _tiled_job, nc, P, 13, 5, dtype, "random")
    tol = 1e-11 if dtype == torch.float64 else 2e-4
    for (a1, a2, t1), (b1, b2, t0) in zip(res["stagger"], res["single"]):
        assert t1 is True and t0 is True
        assert abs(a1 - b1) <= tol * abs(b1), (a1, b1)
        assert abs(a2 - b2) <= tol * abs(b2), (a2, b2)


def test_devicecg_solves_twice_with_different_iterates():
    nc = (5, 6, 7)
    pb = PoissonProblem(Comm(), nc, 3, 1, False, torch.float64, "gpu")
    u = pb.assemble_rhs()
    op = FusedLaplacianGPU(pb, "otf", 4 if fused_supported(pb, 4) else 3)
    cg = DeviceCG(pb)
    x1, x2 = pb.new_vector(), pb.new_vector()
    cg.solve(op, x1, u, 20)
    cg.solve(op, x2, u, 11)
    torch.cuda.synchronize()
    cpu, r20 = _host_cg(nc, 3, 1, False, 20)
    _, r11 = _host_cg(nc, 3, 1, False, 11)
    for x, ref in ((x1, r20), (x2, r11)):
        rel = (cpu.owned(x.cpu()) - cpu.owned(ref)).abs().max().item() / ref.abs().max().item()
        assert rel < 1e-10, rel
    op.close()


def test_phase_profile_single_and_threaded():
    def job(comm):
        pb = PoissonProblem(comm, (4, 16, 18), 3, 1, False, torch.float64, "gpu")
        op = FusedLaplacianGPU(pb, "otf", 3)
        cg = DeviceCG(pb)
        x = pb.new_vector()
        cg.solve(op, x, pb.assemble_rhs(), 4)
        ph = op._rt.profile(3)
        it = cg.it
        op.close()
        return ph, it
    for ranks in (1, 2):
        res = run_threaded(ranks, job)
        # the hidden flags exist for the split (two-stream) schedule only: a
        # rank with ghost planes runs it, a rank without runs serially
        if ranks > 1:
            assert any(isinstance(ph["halo_fwd_hidden"], bool) for ph, _ in res)
        for ph, it in res:
            assert it == 7
            assert ph["iteration"] > 0 and ph["op_interior"] > 0
            assert all(v >= 0 for v in ph.values() if isinstance(v, float))
            assert ph["halo_fwd_hidden"] in (True, False, None)
            for k in ("t_halo_fwd_done", "t_boundary_done", "t_halo_rev_done",
                      "t_op_interior_done"):
                assert ph[k] <= ph["iteration"] + 1e-3, (k, ph)
            if ranks > 1:
                assert ph["halo_fwd"] > 0 and ph["halo_rev"] > 0


def test_bench_entry_point_one_gpu():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--dofs-per-gpu", "2000000",
                        "--steps", "5", "--warmup", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["steps"] == 5
    cfg = line["config"]
    assert cfg["build_flags"]["valid"] and cfg["comm"]["transport"] == "none"
    assert cfg["comm"]["rccl_ranks"] == 1
    assert cfg["phases_ms"]["iteration"] > 0
    assert "gfx950" in cfg["device"]
    assert np.isfinite(cfg["y_norm"]) and cfg["y_norm"] > 0
    assert line["ms_per_step_median"] > 0 and line["ms_per_step_min"] > 0


def _tiled_job(comm, nc, P, nreps, version, dtype, coef, shear=0.0, pert=0.0):
    pb = PoissonProblem(comm, nc, P, 1, False, dtype, "gpu", pert, coef, shear,
                        partition="yz")
    u = pb.assemble_rhs()
    x = pb.new_vector()
    op = FusedLaplacianGPU(pb, "otf", version)
    cg = DeviceCG(pb)
    cg.solve(op, x, u, nreps)
    cg.wait()
    xn = pb.norm(x)
    # a second solve on the same runtime (re-import of the prologue state)
    x2 = pb.new_vector()
    cg.solve(op, x2, u, nreps)
    cg.wait()
    tiled = op._rt.tiled if op._rt is not None else None
    op.close()
    return xn, pb.norm(x2), tiled


@pytest.mark.parametrize("version,P,nc,dtype,coef", [
    (5, 3, (6, 9, 14), torch.float64, "constant"),
    (5, 3, (5, 13, 7), torch.float64, "random"),
    (5, 6, (3, 5, 6), torch.float64, "random"),
    (5, 4, (4, 7, 9), torch.float64, "constant"),
    (5, 5, (3, 6, 5), torch.float64, "constant"),
    (5, 7, (3, 4, 5), torch.float64, "constant"),
    (5, 6, (3, 5, 6), torch.float32, "constant"),
    (5, 3, (5, 9, 10), torch.float32, "random"),
])
@pytest.mark.parametrize("ranks", [1, 4])
def test_tiled_storage_matches_lattice_layout(monkeypatch, version, P, nc, dtype, coef, ranks):
    """The runtime's tiled vector storage (x-march tiles contiguous) against
    the lattice layout: same CG iterate (summation order of r.r differs), on
    1 rank and on 4 threaded ranks (tiled halo pack/unpack and ghost finalize)."""
    monkeypatch.setenv("BDX_TILED", "1")
    got = run_threaded(ranks, _tiled_job, nc, P, 12, version, dtype, coef)
    monkeypatch.setenv("BDX_TILED", "0")
    ref = run_threaded(ranks, _tiled_job, nc, P, 12, version, dtype, coef)
    tol = 1e-11 if dtype == torch.float64 else 2e-4
    for (a1, a2, t1), (b1, b2, t0) in zip(got, ref):
        assert t1 is True and t0 is False
        assert abs(a1 - b1) <= tol * abs(b1), (a1, b1)
        assert abs(a2 - b2) <= tol * abs(b2), (a2, b2)
        assert abs(a1 - a2) <= tol * abs(a1)  # the re-imported solve repeats the first


@pytest.mark.parametrize("P,nc,dtype,coef,pert", [
    (3, (6, 9, 14), torch.float64, "random", 0.15),
    (6, (3, 5, 6), torch.float64, "constant", 0.15),
    (2, (5, 7, 9), torch.float64, "constant", 0.15),
    (3, (5, 9, 10), torch.float32, "constant", 0.15),
    (6, (3, 5, 6), torch.float32, "constant", 0.15),
    (4, (4, 7, 9), torch.float64, "constant", 0.0),
])
@pytest.mark.parametrize("ranks", [1, 4])
def test_tiled_storage_fused3_general(monkeypatch, P, nc, dtype, coef, pert, ranks):
    """fused3 (general trilinear geometry) on the runtime's tiled storage
    against the lattice layout, 1 and 4 threaded ranks (opt-in: BDX_TILED=2;
    an FP32 tile plane that is not a multiple of 16 bytes stays on the
    lattice layout)."""
    monkeypatch.setenv("BDX_TILED", "2")
    got = run_threaded(ranks, _tiled_job, nc, P, 12, 3, dtype, coef, 0.0, pert)
    monkeypatch.setenv("BDX_TILED", "0")
    ref = run_threaded(ranks, _tiled_job, nc, P, 12, 3, dtype, coef, 0.0, pert)
    tol = 1e-11 if dtype == torch.float64 else 2e-4
    for (a1, a2, t1), (b1, b2, t0) in zip(got, ref):
        assert t1 is (dtype == torch.float64 or P % 2 == 0) and t0 is False
        assert abs(a1 - b1) <= tol * abs(b1), (a1, b1)
        assert abs(a2 - b2) <= tol * abs(b2), (a2, b2)


@pytest.mark.parametrize("P,nc,dtype", [(3, (5, 13, 7), torch.float64), (6, (3, 5, 6), torch.float32)])
def test_tiled_update_plain_path_matches(monkeypatch, P, nc, dtype):
    """The tiled update pass's plain kernel (interface partials loaded inside
    their branches; the production path for blocks whose interface buffers
    pass 2^31 bytes) against the prefetching one: same sums in the same order,
    so the CG iterates agree to rounding (the path had no
    test).  BDX_UPD_PLAIN=1 forces it on these small meshes."""
    monkeypatch.setenv("BDX_TILED", "1")
    monkeypatch.setenv("BDX_UPD_PLAIN", "1")
    got = run_threaded(1, _tiled_job, nc, P, 12, 5, dtype, "random")
    monkeypatch.delenv("BDX_UPD_PLAIN")
    ref = run_threaded(1, _tiled_job, nc, P, 12, 5, dtype, "random")
    tol = 1e-13 if dtype == torch.float64 else 1e-6
    for (a1, a2, t1), (b1, b2, t0) in zip(got, ref):
        assert t1 is True and t0 is True
        assert abs(a1 - b1) <= tol * abs(b1), (a1, b1)
        assert abs(a2 - b2) <= tol * abs(b2), (a2, b2)
