"""GPU numerics of the fused structured kernel (lap_fused.h) vs the C++ CPU
operator, the fused CG vs host CG, and multi-rank (in-process threads on one
GPU) partition invariance of the fused CG path."""

import numpy as np
import pytest
import torch

from benchmark_dolfinx_amd.fem.mesh import compute_mesh_size
from benchmark_dolfinx_amd.models.fused import FusedLaplacianGPU
from benchmark_dolfinx_amd.models.poisson import MatFreeLaplacianCPU, PoissonProblem
from benchmark_dolfinx_amd.parallel.comm import Comm, run_threaded
from benchmark_dolfinx_amd.solvers.cg import DeviceCG, cg_solve

pytestmark = pytest.mark.gpu

CASES = [
    # ncells, P, qmode, gauss, perturb, dtype   (tiles: nq=5 -> 2x5, nq=8 -> 2x2, ...)
    ((3, 3, 3), 3, 0, False, 0.0, torch.float64),
    ((4, 5, 7), 3, 1, False, 0.2, torch.float64),
    ((3, 7, 11), 3, 1, True, 0.1, torch.float64),
    ((2, 3, 3), 6, 1, False, 0.15, torch.float64),
    ((3, 2, 5), 6, 0, False, 0.1, torch.float64),
    ((2, 2, 4), 7, 1, False, 0.0, torch.float64),
    ((2, 3, 2), 7, 0, False, 0.2, torch.float64),
    ((9, 10, 17), 1, 1, False, 0.3, torch.float64),
    ((5, 9, 10), 1, 0, False, 0.1, torch.float64),
    ((4, 5, 9), 2, 1, False, 0.1, torch.float64),
    ((4, 5, 9), 2, 0, True if False else False, 0.0, torch.float64),
    ((3, 4, 9), 4, 1, False, 0.2, torch.float64),
    ((3, 3, 8), 5, 1, False, 0.2, torch.float64),
    ((5, 4, 7), 3, 1, False, 0.2, torch.float32),
    ((2, 3, 3), 6, 1, False, 0.1, torch.float32),
    ((6, 9, 11), 3, 1, False, 0.0, torch.float64),
    ((5, 8, 13), 3, 1, True, 0.0, torch.float64),
]


def _tol(dt):
    return 1e-12 if dt == torch.float64 else 3e-5


# (geometry, kernel version, affine fast path allowed)
VARIANTS = [("otf", 1, True), ("stored", 1, True), ("otf", 2, True), ("otf", 2, False),
            ("otf", 3, True), ("otf", 3, False), ("otf", 5, True)]


def _skip_unsupported(pb, version):
    from benchmark_dolfinx_amd.models.fused import fused_supported
    if not fused_supported(pb, version):
        pytest.skip(f"fused{version} does not cover this element / mesh / dtype")


@pytest.mark.parametrize("geometry,version,affine", VARIANTS)
@pytest.mark.parametrize("nc,P,qm,g,pert,dt", CASES)
def test_fused_action_matches_cpu(nc, P, qm, g, pert, dt, geometry, version, affine):
    gpu = PoissonProblem(Comm(), nc, P, qm, g, dt, "gpu", pert)
    _skip_unsupported(gpu, version)
    cpu = PoissonProblem(Comm(), nc, P, qm, g, torch.float64, "cpu", pert)
    rng = np.random.default_rng(3)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    yg = torch.full(gpu.lat.shape, float("nan"), dtype=dt, device=gpu.device)
    FusedLaplacianGPU(gpu, geometry, version, affine).apply(u64.to(gpu.device, dt), yg)
    yg = yg.double().cpu()
    o = cpu.owned
    assert torch.isfinite(o(yg)).all()
    err = (o(yg) - o(yc)).abs().max().item()
    assert err <= _tol(dt) * 50 * max(1.0, yc.abs().max().item()), err


@pytest.mark.parametrize("runtime", ["native", "python"])
@pytest.mark.parametrize("geometry,version,affine", VARIANTS)
@pytest.mark.parametrize("pert", [0.0, 0.1])
def test_fused_cg_matches_host_cg(geometry, version, affine, pert, runtime):
    if version == 1 and runtime == "native":
        pytest.skip("the native runtime drives fused2/3")
    nc = (5, 7, 11)
    gpu = PoissonProblem(Comm(), nc, 3, 1, False, torch.float64, "gpu", pert)
    _skip_unsupported(gpu, version)
    cpu = PoissonProblem(Comm(), nc, 3, 1, False, torch.float64, "cpu", pert)
    xg = gpu.new_vector()
    DeviceCG(gpu).solve(FusedLaplacianGPU(gpu, geometry, version, affine, runtime), xg,
                        gpu.assemble_rhs(), 30)
    xc = cpu.new_vector()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), 30)
    rel = (cpu.owned(xg.cpu()) - cpu.owned(xc)).abs().max().item() / xc.abs().max().item()
    assert rel < 1e-10, rel


def _cg_job(comm, nc, P, nreps, geometry, version=1, pert=0.1, runtime="native"):
    pb = PoissonProblem(comm, nc, P, 1, False, torch.float64, "gpu", pert)
    u = pb.assemble_rhs()
    x = pb.new_vector()
    op = FusedLaplacianGPU(pb, geometry, version, runtime=runtime)
    DeviceCG(pb).solve(op, x, u, nreps)
    y = pb.new_vector()
    op.apply(u, y)
    torch.cuda.synchronize()
    return pb.norm(u), pb.norm(x), pb.norm(y)


@pytest.mark.parametrize("runtime", ["native", "python"])
@pytest.mark.parametrize("pert", [0.0, 0.1])
@pytest.mark.parametrize("version", [1, 2, 3, 5])
@pytest.mark.parametrize("ranks", [2, 4, 8])
def test_fused_partition_invariance_threaded(ranks, version, pert, runtime):
    if version == 5 and pert:
        pytest.skip("fused5 needs axis-aligned box cells")
    if version == 1 and runtime == "native":
        pytest.skip("the native runtime drives fused2/3")
    ref = run_threaded(1, _cg_job, (6, 7, 9), 3, 15, "otf", version, pert, runtime)[0]
    got = run_threaded(ranks, _cg_job, (6, 7, 9), 3, 15, "otf", version, pert, runtime)
    for r in got:
        for a, b in zip(r, ref):
            assert abs(a - b) <= 1e-11 * abs(b), (r, ref)


@pytest.mark.parametrize("version", [1, 2, 3, 5])
def test_fused_golden_and_mat_comp_16(version):
    if version != 3:  # qmode=0 (phi0 == I) is not a fused3 element
        nx = compute_mesh_size(1000, 3)
        pb = PoissonProblem(Comm(), nx, 3, 0, False, torch.float64, "gpu")
        u = pb.assemble_rhs()
        y = pb.new_vector()
        FusedLaplacianGPU(pb, "otf", version).apply(u, y)
        assert abs(pb.norm(y) - 9.912865833415553) < 1e-12
    nx = compute_mesh_size(100000, 3)
    pb = PoissonProblem(Comm(), nx, 3, 1, False, torch.float64, "gpu")
    u = pb.assemble_rhs()
    y = pb.new_vector()
    FusedLaplacianGPU(pb, "otf", version).apply(u, y)
    assert abs(pb.norm(y) - 0.14150257625641838) < 1e-13


@pytest.mark.parametrize("P,nc", [(1, (7, 9, 13)), (2, (5, 9, 9)), (4, (3, 5, 6)), (6, (3, 4, 5)),
                                  (7, (2, 3, 4))])
@pytest.mark.parametrize("pert", [0.0, 0.1])
def test_fused3_cg_all_degrees(P, nc, pert):
    """fused3 CG (incl. the wave-local nq = 4, 8 layouts) against the host CG."""
    gpu = PoissonProblem(Comm(), nc, P, 1, False, torch.float64, "gpu", pert)
    cpu = PoissonProblem(Comm(), nc, P, 1, False, torch.float64, "cpu", pert)
    xg = gpu.new_vector()
    DeviceCG(gpu).solve(FusedLaplacianGPU(gpu, "otf", 3), xg, gpu.assemble_rhs(), 12)
    xc = cpu.new_vector()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), 12)
    rel = (cpu.owned(xg.cpu()) - cpu.owned(xc)).abs().max().item() / xc.abs().max().item()
    assert rel < 1e-10, rel


@pytest.mark.parametrize("kernel", ["fused5", "fused3", "fused2", "v1"])
@pytest.mark.parametrize("nc,P,pert", [((4, 5, 7), 3, 0.0), ((3, 4, 5), 6, 0.1), ((5, 6, 6), 2, 0.0),
                                       ((9, 13, 10), 3, 0.0)])
def test_random_coefficients_gpu(kernel, nc, P, pert):
    """Per-cell random kappa: GPU kernels vs the C++ CPU operator, and CG."""
    from benchmark_dolfinx_amd.driver import make_operator
    gpu = PoissonProblem(Comm(), nc, P, 1, False, torch.float64, "gpu", pert, "random")
    if kernel == "fused5" and not (P >= 3 and pert == 0.0):
        pytest.skip("fused5: P >= 3 parallelepiped cells")
    cpu = PoissonProblem(Comm(), nc, P, 1, False, torch.float64, "cpu", pert, "random")
    rng = np.random.default_rng(5)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    op = make_operator(gpu, kernel)
    yg = gpu.new_vector()
    op.apply(u64.to(gpu.device), yg)
    o = cpu.owned
    err = (o(yg.cpu()) - o(yc)).abs().max().item()
    assert err <= 1e-11 * yc.abs().max().item(), err
    xg = gpu.new_vector()
    DeviceCG(gpu).solve(op, xg, gpu.assemble_rhs(), 10)
    xc = cpu.new_vector()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), 10)
    rel = (o(xg.cpu()) - o(xc)).abs().max().item() / xc.abs().max().item()
    assert rel < 1e-10, rel


@pytest.mark.parametrize("nc,coef", [((4, 8, 8), "constant"), ((8, 4, 16), "random"),
                                     ((16, 8, 4), "constant")])
@pytest.mark.parametrize("shear", [0.5, 0.25])
def test_sheared_parallelepipeds_take_fused3_affine(nc, coef, shear):
    """Parallelepipeds with a full Jacobian (G01/G02/G12 != 0, a sheared
    mesh): fused5 refuses them and the auto choice is fused3's affine
    instance; action vs the C++ CPU operator and CG vs the host CG."""
    from benchmark_dolfinx_amd.driver import make_operator
    from benchmark_dolfinx_amd.models.fused import fused_supported
    gpu = PoissonProblem(Comm(), nc, 3, 1, False, torch.float64, "gpu", 0.0, coef, shear)
    cpu = PoissonProblem(Comm(), nc, 3, 1, False, torch.float64, "cpu", 0.0, coef, shear)
    assert gpu.all_affine and not gpu.all_axis_aligned and not fused_supported(gpu, 5)
    with pytest.raises(ValueError):
        FusedLaplacianGPU(gpu, "otf", 5)
    rng = np.random.default_rng(11)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    op = make_operator(gpu)
    assert op.name == "fused3" and op.geometry == "otf-affine", (op.name, op.geometry)
    yg = gpu.new_vector()
    op.apply(u64.to(gpu.device), yg)
    o = cpu.owned
    err = (o(yg.cpu()) - o(yc)).abs().max().item()
    assert err <= 1e-12 * 50 * yc.abs().max().item(), err
    xg = gpu.new_vector()
    DeviceCG(gpu).solve(op, xg, gpu.assemble_rhs(), 20)
    xc = cpu.new_vector()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), 20)
    rel = (o(xg.cpu()) - o(xc)).abs().max().item() / xc.abs().max().item()
    assert rel < 1e-10, rel
    op.close()


def _cg_job_shear(comm, nc, nreps):
    from benchmark_dolfinx_amd.driver import make_operator
    pb = PoissonProblem(comm, nc, 3, 1, False, torch.float64, "gpu", 0.0, "random", 0.5)
    u = pb.assemble_rhs()
    x = pb.new_vector()
    op = make_operator(pb)
    assert op.name == "fused3", op.name
    DeviceCG(pb).solve(op, x, u, nreps)
    y = pb.new_vector()
    op.apply(u, y)
    torch.cuda.synchronize()
    op.close()
    return pb.norm(u), pb.norm(x), pb.norm(y)


@pytest.mark.parametrize("ranks", [2, 4])
def test_sheared_partition_invariance(ranks):
    ref = run_threaded(1, _cg_job_shear, (8, 8, 16), 12)[0]
    got = run_threaded(ranks, _cg_job_shear, (8, 8, 16), 12)
    for r in got:
        for a, b in zip(r, ref):
            assert abs(a - b) <= 1e-11 * abs(b), (r, ref)


F5_CASES = [
    # ncells, P, qmode, gauss, shear, dtype   (fused5 tiles: P3 4x4, P4 2x4, P>=5 2x2)
    ((3, 5, 6), 3, 1, False, 0.0, torch.float64),
    ((4, 9, 7), 3, 0, False, 0.0, torch.float64),
    ((4, 8, 8), 3, 1, True, 0.375, torch.float64),
    ((3, 3, 5), 4, 1, False, 0.0, torch.float64),
    ((2, 4, 8), 4, 0, False, 0.75, torch.float64),
    ((3, 3, 5), 5, 1, True, 0.0, torch.float64),
    ((2, 4, 4), 5, 1, False, 0.25, torch.float64),
    ((3, 3, 5), 6, 1, False, 0.0, torch.float64),
    ((2, 5, 3), 6, 0, False, 0.0, torch.float64),
    ((4, 2, 4), 6, 1, False, 0.5, torch.float64),
    ((2, 3, 3), 7, 1, False, 0.0, torch.float64),
    ((2, 2, 4), 7, 1, True, 0.125, torch.float64),
    ((4, 5, 7), 3, 1, False, 0.0, torch.float32),
    ((3, 5, 3), 6, 1, False, 0.0, torch.float32),
    ((2, 4, 4), 6, 1, False, 0.25, torch.float32),
    ((3, 3, 3), 7, 1, False, 0.0, torch.float32),
]


@pytest.mark.parametrize("coef", ["constant", "random"])
@pytest.mark.parametrize("nc,P,qm,g,shear,dt", F5_CASES)
def test_fused5_action_and_cg(nc, P, qm, g, shear, dt, coef):
    """fused5 (nodal Kronecker core) on axis-aligned boxes; sheared
    parallelepipeds are refused by fused5 and run fused3's affine instance
    (auto choice); action vs the C++ CPU operator and CG vs the host CG."""
    from benchmark_dolfinx_amd.driver import make_operator
    from benchmark_dolfinx_amd.models.fused import fused_supported
    gpu = PoissonProblem(Comm(), nc, P, qm, g, dt, "gpu", 0.0, coef, shear)
    cpu = PoissonProblem(Comm(), nc, P, qm, g, torch.float64, "cpu", 0.0, coef, shear)
    assert gpu.all_affine and fused_supported(gpu, 5) == (shear == 0.0)
    if shear == 0.0:
        op = FusedLaplacianGPU(gpu, "otf", 5)
        assert op.affine_code == 2
    else:
        op = make_operator(gpu)
        if not (qm == 0 and not g):  # fused3 is the phi0 != I core (else fused2)
            assert op.name == "fused3" and op.geometry == "otf-affine", (op.name, op.geometry)
    rng = np.random.default_rng(17)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    yg = torch.full(gpu.lat.shape, float("nan"), dtype=dt, device=gpu.device)
    op.apply(u64.to(gpu.device, dt), yg)
    o = cpu.owned
    yg = yg.double().cpu()
    assert torch.isfinite(o(yg)).all()
    err = (o(yg) - o(yc)).abs().max().item()
    assert err <= _tol(dt) * 50 * max(1.0, yc.abs().max().item()), err
    if dt == torch.float64:
        xg = gpu.new_vector()
        DeviceCG(gpu).solve(op, xg, gpu.assemble_rhs(), 15)
        xc = cpu.new_vector()
        cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), 15)
        rel = (o(xg.cpu()) - o(xc)).abs().max().item() / xc.abs().max().item()
        assert rel < 1e-10, rel
    op.close()


def _cg_job_f5(comm, nc, P, nreps, shear):
    pb = PoissonProblem(comm, nc, P, 1, False, torch.float64, "gpu", 0.0, "random", shear)
    u = pb.assemble_rhs()
    x = pb.new_vector()
    from benchmark_dolfinx_amd.driver import make_operator
    op = make_operator(pb)  # fused5 on the box, fused3 (affine) when sheared
    assert op.name == ("fused5" if shear == 0.0 else "fused3"), op.name
    DeviceCG(pb).solve(op, x, u, nreps)
    y = pb.new_vector()
    op.apply(u, y)
    torch.cuda.synchronize()
    op.close()
    return pb.norm(u), pb.norm(x), pb.norm(y)


@pytest.mark.parametrize("P,nc", [(6, (4, 4, 8)), (4, (8, 4, 8))])
@pytest.mark.parametrize("shear", [0.0, 0.5])
@pytest.mark.parametrize("ranks", [2, 4])
def test_fused5_partition_invariance(ranks, shear, P, nc):
    ref = run_threaded(1, _cg_job_f5, nc, P, 10, shear)[0]
    got = run_threaded(ranks, _cg_job_f5, nc, P, 10, shear)
    for r in got:
        for a, b in zip(r, ref):
            assert abs(a - b) <= 1e-11 * abs(b), (r, ref)


# ---------------------------------------------------------------- x segments
SEG_CASES = [  # version, P, perturb, dtype
    (5, 3, 0.0, torch.float64), (5, 6, 0.0, torch.float64), (5, 4, 0.0, torch.float32),
    (2, 3, 0.2, torch.float64), (3, 3, 0.2, torch.float64), (3, 5, 0.0, torch.float32),
    (2, 2, 0.1, torch.float64)]


@pytest.mark.parametrize("nseg", ["1", "2", "3", "5", "13", ""])
@pytest.mark.parametrize("kappa", ["constant", "random"])
@pytest.mark.parametrize("version,P,pert,dt", SEG_CASES)
def test_fused_x_segments_cg_and_action(monkeypatch, version, P, pert, dt, nseg, kappa):
    """The fused kernels with the x-march cut into segments (each starting
    with a redundant, unwritten layer) match the CPU operator (action) and
    host CG for any segment count, incl. the automatic choice ("")."""
    monkeypatch.setenv("BDX_SEGMENTS", nseg)
    nc = (13, 5, 6) if P >= 5 else (13, 6, 9)
    gpu = PoissonProblem(Comm(), nc, P, 1, False, dt, "gpu", pert, kappa)
    _skip_unsupported(gpu, version)
    cpu = PoissonProblem(Comm(), nc, P, 1, False, torch.float64, "cpu", pert, kappa)
    op = FusedLaplacianGPU(gpu, "otf", version, affine=pert == 0.0)
    if nseg:
        n = int(nseg)
        assert op.nseg == -(-13 // -(-13 // n)), (op.nseg, n)
    rng = np.random.default_rng(5)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    yg = torch.full(gpu.lat.shape, float("nan"), dtype=dt, device=gpu.device)
    op.apply(u64.to(gpu.device, dt), yg)
    o = cpu.owned
    err = (o(yg.double().cpu()) - o(yc)).abs().max().item()
    assert err <= _tol(dt) * 50 * max(1.0, yc.abs().max().item()), err
    xg = gpu.new_vector()
    DeviceCG(gpu).solve(op, xg, gpu.assemble_rhs(), 25)
    xc = cpu.new_vector()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), 25)
    rel = (o(xg.double().cpu()) - o(xc)).abs().max().item() / xc.abs().max().item()
    assert rel < (1e-10 if dt == torch.float64 else 2e-4), rel
    op.close()


@pytest.mark.parametrize("nseg", ["2", "4"])
@pytest.mark.parametrize("ranks", [2, 4])
@pytest.mark.parametrize("version,pert", [(5, 0.0), (3, 0.1)])
def test_fused_x_segments_partition_invariance(monkeypatch, version, pert, nseg, ranks):
    monkeypatch.setenv("BDX_SEGMENTS", nseg)
    ref = run_threaded(1, _cg_job, (11, 14, 17), 3, 12, "otf", version, pert, "native")[0]
    got = run_threaded(ranks, _cg_job, (11, 14, 17), 3, 12, "otf", version, pert, "native")
    for r in got:
        for a, b in zip(r, ref):
            assert abs(a - b) <= 1e-11 * abs(b), (r, ref)


@pytest.mark.parametrize("nc,P,dt", [((4, 5, 7), 3, torch.float64), ((3, 7, 11), 3, torch.float64),
                                     ((2, 3, 3), 6, torch.float64), ((3, 3, 8), 5, torch.float64),
                                     ((5, 4, 7), 3, torch.float32), ((2, 3, 3), 6, torch.float32),
                                     ((3, 4, 9), 4, torch.float64), ((7, 9, 13), 1, torch.float64),
                                     ((2, 3, 4), 7, torch.float64)])
@pytest.mark.parametrize("coef", ["constant", "random"])
def test_fused3_x_trilinear_instance(nc, P, dt, coef):
    """fused3's x-trilinear instance (AFF = 2: y/z on the lattice, x perturbed
    as src/mesh.cpp:199-207) is auto-selected on perturbed meshes and matches
    the CPU operator and the general trilinear instance; a sheared perturbed
    mesh keeps the general instance."""
    from benchmark_dolfinx_amd.driver import make_operator
    gpu = PoissonProblem(Comm(), nc, P, 1, False, dt, "gpu", 0.2, coef)
    _skip_unsupported(gpu, 3)
    cpu = PoissonProblem(Comm(), nc, P, 1, False, torch.float64, "cpu", 0.2, coef)
    op = make_operator(gpu)
    assert op.name == "fused3" and op.geometry == "otf-xtrilinear" and op.affine_code == 2
    gen = make_operator(gpu, "fused3", "otf-general")
    assert gen.geometry == "otf-general" and gen.affine_code == 0
    rng = np.random.default_rng(11)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    o = cpu.owned
    scale = max(1.0, yc.abs().max().item())
    for k in (op, gen):
        yg = torch.full(gpu.lat.shape, float("nan"), dtype=dt, device=gpu.device)
        k.apply(u64.to(gpu.device, dt), yg)
        yg = yg.double().cpu()
        assert torch.isfinite(o(yg)).all()
        err = (o(yg) - o(yc)).abs().max().item()
        assert err <= _tol(dt) * 50 * scale, (k.geometry, err)
    if dt == torch.float64:
        xg = gpu.new_vector()
        DeviceCG(gpu).solve(op, xg, gpu.assemble_rhs(), 12)
        xc = cpu.new_vector()
        cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), 12)
        rel = (o(xg.cpu()) - o(xc)).abs().max().item() / xc.abs().max().item()
        assert rel < 1e-10, rel
    sh = PoissonProblem(Comm(), nc, P, 1, False, dt, "gpu", 0.2, coef, 0.3)
    assert make_operator(sh).geometry == "otf-general"


@pytest.mark.parametrize("P,nc", [(6, (3, 4, 5)), (6, (2, 5, 3)), (7, (2, 3, 4))])
@pytest.mark.parametrize("pert", [0.0, 0.2])
@pytest.mark.parametrize("coef", ["constant", "random"])
def test_fused3_fp32_q6_q7(P, nc, pert, coef):
    """fused3 in FP32 at P = 6 (y / z stages on v_mfma_f32_16x16x4_f32 for the
    parallelepiped and x-trilinear instances) and P = 7 (VALU): action vs the
    FP64 C++ CPU operator, CG vs the FP64 host CG (FP32 tolerances)."""
    gpu = PoissonProblem(Comm(), nc, P, 1, False, torch.float32, "gpu", pert, coef)
    _skip_unsupported(gpu, 3)
    cpu = PoissonProblem(Comm(), nc, P, 1, False, torch.float64, "cpu", pert, coef)
    op = FusedLaplacianGPU(gpu, "otf", 3)
    assert op.affine_code == (1 if pert == 0.0 else 2)
    rng = np.random.default_rng(21)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    yg = torch.full(gpu.lat.shape, float("nan"), dtype=torch.float32, device=gpu.device)
    op.apply(u64.to(gpu.device, torch.float32), yg)
    o = cpu.owned
    yg = yg.double().cpu()
    assert torch.isfinite(o(yg)).all()
    err = (o(yg) - o(yc)).abs().max().item()
    assert err <= _tol(torch.float32) * 50 * max(1.0, yc.abs().max().item()), err
    xg = gpu.new_vector()
    DeviceCG(gpu).solve(op, xg, gpu.assemble_rhs(), 15)
    xc = cpu.new_vector()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, cpu.assemble_rhs(), 15)
    rel = (o(xg.double().cpu()) - o(xc)).abs().max().item() / xc.abs().max().item()
    assert rel < 2e-4, rel
    op.close()


@pytest.mark.parametrize("ranks", [2, 4])
def test_fused3_x_trilinear_partition_invariance(ranks):
    ref = run_threaded(1, _cg_job, (6, 7, 9), 3, 15, "otf", 3, 0.15)[0]
    for r in run_threaded(ranks, _cg_job, (6, 7, 9), 3, 15, "otf", 3, 0.15):
        for a, b in zip(r, ref):
            assert abs(a - b) <= 1e-11 * abs(b), (r, ref)


@pytest.mark.parametrize("nc,P,qm,g,dt", [((4, 5, 7), 3, 0, False, torch.float64),
                                         ((2, 3, 3), 6, 0, False, torch.float64),
                                         ((5, 4, 7), 3, 0, False, torch.float32),
                                         ((3, 7, 11), 2, 1, True, torch.float64)])
def test_fused2_x_trilinear_instance(nc, P, qm, g, dt):
    """fused2's x-trilinear instance (qmode=0 GLL collocation, or forced)
    against the CPU operator and fused2's general instance."""
    gpu = PoissonProblem(Comm(), nc, P, qm, g, dt, "gpu", 0.2)
    _skip_unsupported(gpu, 2)
    cpu = PoissonProblem(Comm(), nc, P, qm, g, torch.float64, "cpu", 0.2)
    xt = FusedLaplacianGPU(gpu, "otf", 2)
    gen = FusedLaplacianGPU(gpu, "otf", 2, affine=False)
    assert xt.affine_code == 2 and xt.geometry == "otf-xtrilinear" and gen.affine_code == 0
    rng = np.random.default_rng(12)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    o = cpu.owned
    scale = max(1.0, yc.abs().max().item())
    for k in (xt, gen):
        yg = torch.full(gpu.lat.shape, float("nan"), dtype=dt, device=gpu.device)
        k.apply(u64.to(gpu.device, dt), yg)
        yg = yg.double().cpu()
        err = (o(yg) - o(yc)).abs().max().item()
        assert err <= _tol(dt) * 50 * scale, (k.geometry, err)


def test_segment_model_choices():
    """The fractional-round segment model (lap_fused2.h fused_choose_segments)
    on the headline tile counts: fused5 Q6 (66 x 66 tiles, 132 layers) splits
    the march (whole rounds kept S = 1), fused3's x-trilinear instance takes at
    least 2 segments, and no choice exceeds the layer count (profiles/r2_segments.md)."""
    from benchmark_dolfinx_amd.ops import native
    lib = native.hip()
    assert lib.bdx_fused5_segments_f64_p6(2, 66 * 66, 132) >= 2
    assert lib.bdx_fused3_segments_f64_p6(2, 8, 66 * 66, 132) >= 2
    assert 1 <= lib.bdx_fused3_segments_f64_p3(2, 5, 2, 4) <= 4
    for s in (lib.bdx_fused5_segments_f64_p3(2, 56 * 56, 222),
              lib.bdx_fused3_segments_f64_p3(0, 5, 112 * 45, 222)):
        assert 1 <= s <= 16
