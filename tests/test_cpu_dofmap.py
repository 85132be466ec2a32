"""The reference data model on the CPU platform (DofmapLaplacianCPU: explicit
cell -> dof map, G stored per cell in the reference layout or computed per
point, atomic scatter; the reference's own MatFreeLaplacianCPU path,
src/laplacian.hpp:450-771) against the lattice CPU operator, on one and on
several in-process ranks (the overlapped interior / boundary split)."""

import numpy as np
import pytest
import torch

from benchmark_dolfinx_amd.driver import make_operator
from benchmark_dolfinx_amd.models.poisson import MatFreeLaplacianCPU, PoissonProblem
from benchmark_dolfinx_amd.models.unstructured import DofmapLaplacianCPU
from benchmark_dolfinx_amd.parallel.comm import Comm, run_threaded
from benchmark_dolfinx_amd.solvers.cg import cg_solve

CASES = [
    # ncells, P, qmode, gauss, perturb, dtype, kappa
    ((3, 3, 3), 3, 0, False, 0.0, torch.float64, "constant"),
    ((4, 5, 3), 3, 1, False, 0.2, torch.float64, "random"),
    ((3, 4, 2), 2, 1, True, 0.1, torch.float64, "constant"),
    ((2, 3, 3), 6, 1, False, 0.15, torch.float64, "random"),
    ((2, 2, 3), 7, 1, False, 0.0, torch.float64, "constant"),
    ((5, 4, 3), 1, 1, False, 0.3, torch.float64, "constant"),
    ((3, 2, 2), 5, 1, False, 0.1, torch.float64, "random"),
    ((4, 3, 3), 3, 1, False, 0.2, torch.float32, "constant"),
]


@pytest.mark.parametrize("geometry", ["stored", "otf"])
@pytest.mark.parametrize("nc,P,qm,g,pert,dt,kappa", CASES)
def test_cpu_dofmap_matches_lattice_operator(nc, P, qm, g, pert, dt, kappa, geometry):
    pb = PoissonProblem(Comm(), nc, P, qm, g, dt, "cpu", pert, kappa)
    rng = np.random.default_rng(3)
    u = torch.from_numpy(rng.standard_normal(pb.lat.shape)).to(dt)
    y_ref, y = pb.new_vector(), pb.new_vector()
    MatFreeLaplacianCPU(pb).apply(u, y_ref)
    op = make_operator(pb, "dofmap", geometry)
    assert isinstance(op, DofmapLaplacianCPU) and op.geometry == f"dofmap-{geometry}"
    op.apply(u, y)
    tol = 1e-12 if dt == torch.float64 else 2e-5
    err = (pb.owned(y) - pb.owned(y_ref)).abs().max().item()
    assert err <= tol * 10 * max(1.0, pb.owned(y_ref).abs().max().item()), err


@pytest.mark.parametrize("R", [2, 4])
def test_cpu_dofmap_partition_invariance(R):
    nx = (5, 6, 4)

    def body(comm):
        pb = PoissonProblem(comm, nx, 3, 1, False, torch.float64, "cpu", 0.1, "random")
        u = pb.assemble_rhs()
        x = pb.new_vector()
        cg_solve(DofmapLaplacianCPU(pb), pb, x, u, 6)
        return pb.norm(x), len(DofmapLaplacianCPU(pb).outer)

    ref = body(Comm())[0]
    got = run_threaded(R, body)
    assert any(nb > 0 for _, nb in got)  # the boundary (post-exchange) cells ran
    for xn, _ in got:
        assert abs(xn - ref) <= 1e-11 * abs(ref), (xn, ref)
