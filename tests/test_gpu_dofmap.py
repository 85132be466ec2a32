"""GPU tests of the unstructured (dofmap) operator, csrc/hip/lap_dofmap.h:
against the C++ CPU operator (all degrees, both quadrature modes, perturbed
and random-coefficient meshes, FP64 / FP32, on-the-fly and stored G),
equivariance under arbitrary dof / cell / vertex renumbering, multi-rank
partition invariance with the overlapped halo schedule, and CG."""

import numpy as np
import pytest
import torch

from benchmark_dolfinx_amd.driver import make_operator
from benchmark_dolfinx_amd.models.poisson import MatFreeLaplacianCPU, PoissonProblem
from benchmark_dolfinx_amd.models.unstructured import DofmapLaplacianGPU
from benchmark_dolfinx_amd.parallel.comm import Comm, run_threaded
from benchmark_dolfinx_amd.solvers.cg import DeviceCG, cg_solve

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["valu", "mfma"], autouse=True)
def dofmap_kernel(request):
    """Every test runs on both FP64 operator kernels of the data model: the
    line-per-lane VALU kernel (lap_dofmap.h) and the MFMA one
    (lap_dofmfma.h); FP32 always takes the VALU kernel."""
    from benchmark_dolfinx_amd.ops import native
    lib = native.hip()
    lib.bdx_dofmap_set_mfma(1 if request.param == "mfma" else 0)
    yield request.param
    lib.bdx_dofmap_set_mfma(-1)

CASES = [
    # ncells, P, qmode, gauss, perturb, dtype, kappa
    ((3, 3, 3), 3, 0, False, 0.0, torch.float64, "constant"),
    ((4, 5, 3), 3, 1, False, 0.2, torch.float64, "random"),
    ((3, 4, 2), 2, 1, True, 0.1, torch.float64, "constant"),
    ((2, 3, 3), 6, 1, False, 0.15, torch.float64, "random"),
    ((2, 2, 3), 7, 1, False, 0.0, torch.float64, "constant"),
    ((5, 4, 3), 1, 1, False, 0.3, torch.float64, "constant"),
    ((3, 3, 4), 4, 0, False, 0.0, torch.float64, "constant"),
    ((3, 2, 2), 5, 1, False, 0.1, torch.float64, "random"),
    ((4, 3, 3), 3, 1, False, 0.2, torch.float32, "constant"),
    ((2, 3, 2), 6, 1, False, 0.1, torch.float32, "random"),
]


def _tol(dt):
    return 1e-12 if dt == torch.float64 else 2e-5


@pytest.mark.parametrize("geometry", ["otf", "stored"])
@pytest.mark.parametrize("nc,P,qm,g,pert,dt,kappa", CASES)
def test_dofmap_matches_cpu(nc, P, qm, g, pert, dt, kappa, geometry):
    gpu = PoissonProblem(Comm(), nc, P, qm, g, dt, "gpu", pert, kappa)
    cpu = PoissonProblem(Comm(), nc, P, qm, g, torch.float64, "cpu", pert, kappa)
    rng = np.random.default_rng(2)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    yg = gpu.new_vector()
    op = make_operator(gpu, "dofmap", geometry)
    assert isinstance(op, DofmapLaplacianGPU)
    op.apply(u64.to(gpu.device, dt), yg)
    err = (cpu.owned(yg.double().cpu()) - cpu.owned(yc)).abs().max().item()
    assert err <= _tol(dt) * 50 * max(1.0, yc.abs().max().item()), err


@pytest.mark.parametrize("P,pert", [(3, 0.2), (6, 0.1)])
def test_dofmap_equivariant_under_renumbering(P, pert):
    pb = PoissonProblem(Comm(), (3, 4, 3), P, 1, False, torch.float64, "gpu", pert, "random")
    op = DofmapLaplacianGPU(pb)
    rng = np.random.default_rng(7)
    u = torch.from_numpy(rng.standard_normal(pb.lat.nstore)).to(pb.device)
    y = pb.new_vector()
    op.apply(u.view(pb.lat.shape), y)
    m = op.mesh
    dp = rng.permutation(m.ndofs)
    cp = rng.permutation(m.ncells)
    vp = rng.permutation(m.coords.shape[0])
    op2 = DofmapLaplacianGPU(pb, mesh=m.renumbered(dp, cp, vp))
    dpt = torch.from_numpy(dp).to(pb.device)
    u2 = torch.empty_like(u)
    u2[dpt] = u  # u2[dp[i]] = u[i]
    y2 = torch.zeros_like(u)
    op2.apply(u2, y2)
    ref = y.reshape(-1)
    got = y2[dpt]
    assert (got - ref).abs().max().item() <= 1e-12 * ref.abs().max().item()


def _cg_job(comm, nc, P, nits, pert, runtime="native"):
    pb = PoissonProblem(comm, nc, P, 1, False, torch.float64, "gpu", pert, "random")
    u = pb.assemble_rhs()
    x = pb.new_vector()
    op = DofmapLaplacianGPU(pb, runtime=runtime)
    cg = DeviceCG(pb)
    cg.solve(op, x, u, nits)
    cg.wait()
    rt = op._rt
    info = (rt.transport, rt.overlap) if rt is not None else None
    op.close()
    return pb.norm(x), len(op.mesh.boundary_cells), info


@pytest.mark.parametrize("runtime", ["native", "python"])
@pytest.mark.parametrize("ranks", [2, 4])
def test_dofmap_partition_invariance_threaded(ranks, runtime):
    """Thread ranks on one GPU; `native`: the C++ loop (DofCGRuntime) with its
    split schedule (interior cells || forward exchange -> boundary cells ->
    reverse send), `python`: the same kernels driven with torch collectives."""
    ref = run_threaded(1, _cg_job, (5, 6, 7), 3, 12, 0.15)[0][0]
    got = run_threaded(ranks, _cg_job, (5, 6, 7), 3, 12, 0.15, runtime)
    assert any(nb > 0 for _, nb, _ in got)  # the overlapped boundary pass ran
    for xn, _, info in got:
        assert abs(xn - ref) <= 1e-11 * abs(ref), (xn, ref)
        if runtime == "native":
            assert info is not None and info[0] == "thread", info
    if runtime == "native":
        assert any(info[1] for _, _, info in got)  # the two-stream schedule ran


@pytest.mark.parametrize("runtime", ["native", "python"])
@pytest.mark.parametrize("nc,P,qm,geometry,dt,kappa", [
    ((4, 3, 5), 3, 1, "stored", torch.float64, "constant"),
    ((4, 3, 5), 3, 1, "otf", torch.float64, "random"),
    ((3, 3, 4), 4, 0, "stored", torch.float64, "constant"),
    ((2, 2, 3), 6, 1, "stored", torch.float64, "random"),
    ((2, 2, 2), 7, 1, "otf", torch.float64, "constant"),
    ((3, 4, 3), 3, 1, "stored", torch.float32, "constant"),
])
def test_dofmap_cg_matches_host_cg(nc, P, qm, geometry, dt, kappa, runtime):
    """The fused dofmap CG iteration (p update, lagged x, p.Ap element dots
    and the r / y update pass), in the native C++ loop and driven from
    Python, against the host CG on the CPU operator."""
    gpu = PoissonProblem(Comm(), nc, P, qm, False, dt, "gpu", 0.1, kappa)
    cpu = PoissonProblem(Comm(), nc, P, qm, False, torch.float64, "cpu", 0.1, kappa)
    ug, uc = gpu.assemble_rhs(), cpu.assemble_rhs()
    xg, xc = gpu.new_vector(), cpu.new_vector()
    op = DofmapLaplacianGPU(gpu, geometry, runtime=runtime)
    cg = DeviceCG(gpu)
    cg.start(op, xg, ug)
    assert (op._rt is not None) == (runtime == "native")
    cg.iterate(7)   # two calls: the lagged x update is flushed and resumed
    ms = cg.iterate_timed(13)  # per-step calls, one flush at the end (bench path)
    assert len(ms) == 13
    torch.cuda.synchronize()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, uc, 20, 0.0)
    tol = 1e-10 if dt == torch.float64 else 2e-4
    xo, xr = cpu.owned(xg.double().cpu()), cpu.owned(xc)
    assert (xo - xr).abs().max().item() <= tol * xr.abs().max().item()


@pytest.mark.parametrize("first", [6, 7])
def test_dofmap_native_second_solve_after_even_and_odd_counts(first):
    """the native runtime's y ping-pong leaves the caller's y
    holding A p of the last even iteration.  A second solve on the same
    operator / DeviceCG (the reset path) after an even and after an odd
    iteration count must equal a fresh solve, even with cg.y overwritten in
    between (cg_start zeroes it; nothing may rely on it after iterate)."""
    pb = PoissonProblem(Comm(), (4, 3, 5), 3, 1, False, torch.float64, "gpu", 0.1, "random")
    u = pb.assemble_rhs()
    op = DofmapLaplacianGPU(pb, "stored")
    cg = DeviceCG(pb)
    x1 = pb.new_vector()
    cg.solve(op, x1, u, first)
    cg.wait()
    assert op._rt is not None
    cg.y.fill_(1e300)  # garbage in the caller's y between the solves
    x2 = pb.new_vector()
    cg.solve(op, x2, u, 9)
    cg.wait()
    op.close()
    ref_op = DofmapLaplacianGPU(pb, "stored")
    ref_cg = DeviceCG(pb)
    x3 = pb.new_vector()
    ref_cg.solve(ref_op, x3, u, 9)
    ref_cg.wait()
    ref_op.close()
    torch.cuda.synchronize()
    d = (pb.owned(x2) - pb.owned(x3)).abs().max().item()
    assert d <= 1e-11 * pb.owned(x3).abs().max().item(), d  # float atomics: rounding only
