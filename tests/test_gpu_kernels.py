"""GPU numerics: every HIP kernel against the C++/numpy references.

All tests run in one process on the GPU box (`pytest -m gpu`).
"""

import numpy as np
import pytest
import torch

from benchmark_dolfinx_amd.fem.mesh import compute_mesh_size
from benchmark_dolfinx_amd.models.poisson import (CSROperator, MatFreeLaplacianCPU,
                                                  MatFreeLaplacianGPU, PoissonProblem)
from benchmark_dolfinx_amd.parallel.comm import Comm
from benchmark_dolfinx_amd.solvers.cg import DeviceCG, cg_solve

pytestmark = pytest.mark.gpu

CASES = [
    # ncells, P, qmode, gauss, perturb, dtype
    ((3, 3, 3), 3, 0, False, 0.0, torch.float64),
    ((4, 5, 3), 3, 1, False, 0.2, torch.float64),
    ((3, 4, 2), 2, 1, True, 0.1, torch.float64),
    ((2, 3, 3), 6, 1, False, 0.15, torch.float64),
    ((2, 2, 3), 7, 1, False, 0.0, torch.float64),
    ((5, 4, 3), 1, 1, False, 0.3, torch.float64),
    ((3, 3, 4), 4, 0, False, 0.0, torch.float64),
    ((4, 3, 3), 3, 1, False, 0.2, torch.float32),
    ((2, 3, 2), 6, 1, False, 0.1, torch.float32),
]


def _pair(nc, P, qm, g, pert, dt):
    gpu = PoissonProblem(Comm(), nc, P, qm, g, dt, "gpu", pert)
    cpu = PoissonProblem(Comm(), nc, P, qm, g, torch.float64, "cpu", pert)
    return gpu, cpu


def _tol(dt):
    return 1e-12 if dt == torch.float64 else 2e-5


@pytest.mark.parametrize("nc,P,qm,g,pert,dt", CASES)
def test_rhs_matches_cpu(nc, P, qm, g, pert, dt):
    gpu, cpu = _pair(nc, P, qm, g, pert, dt)
    bg = gpu.assemble_rhs().double().cpu()
    bc = cpu.assemble_rhs()
    err = (cpu.owned(bg) - cpu.owned(bc)).abs().max().item()
    assert err <= _tol(dt) * max(1.0, bc.abs().max().item())


@pytest.mark.parametrize("geometry", ["stored", "otf"])
@pytest.mark.parametrize("nc,P,qm,g,pert,dt", CASES)
def test_v1_stiffness_matches_cpu(nc, P, qm, g, pert, dt, geometry):
    gpu, cpu = _pair(nc, P, qm, g, pert, dt)
    rng = np.random.default_rng(1)
    u64 = torch.from_numpy(rng.standard_normal(cpu.lat.shape))
    yc = cpu.new_vector()
    MatFreeLaplacianCPU(cpu).apply(u64, yc)
    ug = u64.to(gpu.device, dt)
    yg = gpu.new_vector()
    MatFreeLaplacianGPU(gpu, geometry).apply(ug, yg)
    yg = yg.double().cpu()
    err = (cpu.owned(yg) - cpu.owned(yc)).abs().max().item()
    assert err <= _tol(dt) * 50 * max(1.0, yc.abs().max().item())


def test_csr_spmv_matches_cpu():
    gpu, cpu = _pair((4, 3, 5), 3, 1, False, 0.1, torch.float64)
    u = cpu.assemble_rhs()
    A_c = CSROperator(cpu)
    A_g = CSROperator(gpu)
    zc, zg = cpu.new_vector(), gpu.new_vector()
    A_c.apply(u, zc)
    A_g.apply(u.to(gpu.device), zg)
    assert torch.allclose(cpu.owned(zg.cpu()), cpu.owned(zc), rtol=1e-13, atol=1e-13)


def test_blas_kernels():
    pb = PoissonProblem(Comm(), (5, 6, 7), 3, 1, False, torch.float64, "gpu")
    k = pb.kernels
    g = torch.Generator(device="cpu").manual_seed(0)
    vecs = [torch.randn(pb.lat.shape, generator=g, dtype=torch.float64).to(pb.device)
            for _ in range(4)]
    x, r, p, y = vecs
    scal = torch.zeros(8, dtype=torch.float64, device=pb.device)
    part = torch.zeros(k.npart, dtype=torch.float64, device=pb.device)
    k.dot(p, y, part, scal, 2)
    ref = (pb.owned(p) * pb.owned(y)).sum().item()
    assert abs(scal[2].item() - ref) < 1e-10 * abs(ref) + 1e-12
    scal[0] = 3.0
    x0, r0 = x.clone(), r.clone()
    k.cg_update(x, r, p, y, scal, 0, 2, 1, part)
    alpha = 3.0 / scal[2].item()
    o = pb.owned
    assert torch.allclose(o(x), o(x0) + alpha * o(p), rtol=1e-14, atol=1e-14)
    assert torch.allclose(o(r), o(r0) - alpha * o(y), rtol=1e-14, atol=1e-13)
    assert abs(scal[1].item() - (o(r) ** 2).sum().item()) < 1e-9
    p0 = p.clone()
    k.p_update(p, r, scal, 1, 0)
    beta = scal[1].item() / 3.0
    assert torch.allclose(o(p), beta * o(p0) + o(r), rtol=1e-13, atol=1e-13)
    out = pb.new_vector()
    k.axpy(out, -1.0, y, r)
    assert torch.allclose(o(out), o(r) - o(y))


def test_device_cg_matches_host_cg():
    gpu, cpu = _pair((4, 4, 5), 3, 1, False, 0.1, torch.float64)
    ug = gpu.assemble_rhs()
    uc = cpu.assemble_rhs()
    xg = gpu.new_vector()
    DeviceCG(gpu).solve(MatFreeLaplacianGPU(gpu, "otf"), xg, ug, 25)
    xc = cpu.new_vector()
    cg_solve(MatFreeLaplacianCPU(cpu), cpu, xc, uc, 25)
    assert abs(gpu.norm(xg) - cpu.norm(xc)) < 1e-10 * cpu.norm(xc)


def test_golden_1000_dofs_gpu():
    nx = compute_mesh_size(1000, 3)
    pb = PoissonProblem(Comm(), nx, 3, 0, False, torch.float64, "gpu")
    u = pb.assemble_rhs()
    y = pb.new_vector()
    MatFreeLaplacianGPU(pb, "stored").apply(u, y)
    assert abs(pb.norm(y) - 9.912865833415553) < 1e-12


def test_mat_comp_16_norms_gpu():
    nx = compute_mesh_size(100000, 3)
    pb = PoissonProblem(Comm(), nx, 3, 1, False, torch.float64, "gpu")
    u = pb.assemble_rhs()
    y = pb.new_vector()
    MatFreeLaplacianGPU(pb, "otf").apply(u, y)
    assert abs(pb.norm(u) - 0.6895773850559623) < 1e-13
    assert abs(pb.norm(y) - 0.14150257625641838) < 1e-13
