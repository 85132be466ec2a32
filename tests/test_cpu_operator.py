"""CPU path (C++ host library) against the numpy oracles and the reference's
published numbers (src/test_output.py:19, examples/mat_comp-16.json,
examples/Q3-300M.json, examples/Q6-500M.json)."""

import numpy as np
import pytest
import torch

import oracle
from benchmark_dolfinx_amd.fem.mesh import compute_mesh_size, make_local_lattice, vertex_coordinates
from benchmark_dolfinx_amd.models.poisson import CSROperator, MatFreeLaplacianCPU, PoissonProblem
from benchmark_dolfinx_amd.parallel.comm import Comm, run_threaded
from benchmark_dolfinx_amd.solvers.cg import cg_solve


def _problem(nc, P, qm=1, g=False, pert=0.0, comm=None, dt=torch.float64):
    return PoissonProblem(comm or Comm(), nc, P, qm, g, dt, "cpu", pert)


def test_ci_golden_1000_dofs():
    """The reference CI check: --ndofs=1000 --degree=3 --qmode=0 --nreps=1."""
    pb = _problem(compute_mesh_size(1000, 3), 3, 0)
    assert pb.ndofs_global == 1000
    u = pb.assemble_rhs()
    y = pb.new_vector()
    MatFreeLaplacianCPU(pb).apply(u, y)
    assert abs(pb.norm(y) - 9.912865833415553) < 1e-12
    assert abs(pb.norm(u) - 7.879507448215886) < 1e-12
    z = pb.new_vector()
    CSROperator(pb).apply(u, z)
    assert pb.norm(z - y) < 1e-13 * pb.norm(y)


def test_mat_comp_16_published_norms():
    """examples/mat_comp-16.json: Q3 qmode=1, 100048 dofs, 1 action."""
    nx = compute_mesh_size(100000, 3)
    pb = _problem(nx, 3, 1)
    assert pb.ndofs_global == 100048 and pb.ncells_global == 3468
    u = pb.assemble_rhs()
    y = pb.new_vector()
    MatFreeLaplacianCPU(pb).apply(u, y)
    assert abs(pb.norm(u) - 0.6895773850559623) < 1e-13
    assert abs(pb.norm(y) - 0.14150257625641838) < 1e-13
    z = pb.new_vector()
    CSROperator(pb).apply(u, z)
    assert abs(pb.norm(z) - 0.14150257625641852) < 1e-13
    assert pb.norm(z - y) / pb.norm(z) < 1e-13


CASES = [
    ((2, 3, 2), 1, 1, False, 0.0),
    ((2, 2, 3), 2, 0, False, 0.2),
    ((3, 2, 2), 2, 1, True, 0.1),
    ((2, 2, 2), 3, 1, False, 0.25),
    ((2, 2, 2), 4, 0, False, 0.1),
    ((1, 2, 2), 5, 1, False, 0.1),
    ((2, 1, 2), 6, 1, True, 0.0),
    ((1, 2, 1), 7, 0, False, 0.2),
    ((1, 1, 2), 7, 1, False, 0.0),
]


def _global_vertices(nc, pert):
    return vertex_coordinates(make_local_lattice(0, 1, nc, 1), pert)


@pytest.mark.parametrize("nc,P,qm,g,pert", CASES)
def test_cpu_operator_vs_oracle(nc, P, qm, g, pert):
    pb = _problem(nc, P, qm, g, pert)
    ref = oracle.box_model(nc, P, qm, g, vertices=_global_vertices(nc, pert))
    u = pb.assemble_rhs()
    assert np.allclose(pb.to_global_array(u), ref["u"], rtol=1e-12, atol=1e-12)
    y = pb.new_vector()
    MatFreeLaplacianCPU(pb).apply(u, y)
    ya = pb.to_global_array(y)
    assert np.abs(ya - ref["y"]).max() <= 1e-11 * max(1, np.abs(ref["y"]).max())
    # random input
    rng = np.random.default_rng(7)
    xg = rng.standard_normal(ref["u"].size)
    x = pb.new_vector()
    gi = pb.lat.global_indices()
    x[:, :, : pb.lat.L[2]] = torch.from_numpy(xg[gi])
    MatFreeLaplacianCPU(pb).apply(x, y)
    yr = ref["apply"](xg)
    assert np.abs(pb.to_global_array(y) - yr).max() <= 1e-11 * max(1, np.abs(yr).max())
    # assembled CSR agrees
    z = pb.new_vector()
    CSROperator(pb).apply(x, z)
    assert np.abs(pb.to_global_array(z) - yr).max() <= 1e-11 * max(1, np.abs(yr).max())


def test_cpu_float32():
    nc = (3, 2, 4)
    pb = _problem(nc, 3, 1, dt=torch.float32)
    ref = oracle.box_model(nc, 3, 1)
    u = pb.assemble_rhs()
    y = pb.new_vector()
    MatFreeLaplacianCPU(pb).apply(u, y)
    ya = pb.to_global_array(y)
    assert np.abs(ya - ref["y"]).max() <= 1e-5 * np.abs(ref["y"]).max()


@pytest.mark.parametrize("qm", [0, 1])
def test_cg_vs_oracle(qm):
    nc, P = (3, 3, 2), 2
    pb = _problem(nc, P, qm, pert=0.1)
    ref = oracle.box_model(nc, P, qm, vertices=_global_vertices(nc, 0.1))
    u = pb.assemble_rhs()
    x = pb.new_vector()
    cg_solve(MatFreeLaplacianCPU(pb), pb, x, u, 7)
    xr = oracle.cg_model(ref["apply"], ref["u"], 7)
    assert np.abs(pb.to_global_array(x) - xr).max() <= 1e-10 * np.abs(xr).max()


@pytest.mark.parametrize("nc,P,qm", [((3, 3, 3), 3, 0), ((12, 17, 17), 3, 1), ((4, 3, 5), 6, 1)])
def test_kron_oracle_small(nc, P, qm):
    """The closed form agrees with the direct model."""
    un, yn = oracle.kron_norms(nc, P, qm)
    if np.prod(nc) <= 27 * 4:
        ref = oracle.box_model(nc, P, qm)
        assert abs(un - np.linalg.norm(ref["u"])) < 1e-12 * un
        assert abs(yn - np.linalg.norm(ref["y"])) < 1e-11 * yn
    if nc == (3, 3, 3):
        assert abs(yn - 9.912865833415553) < 1e-12
    if nc == (12, 17, 17):
        assert abs(un - 0.6895773850559623) < 1e-13
        assert abs(yn - 0.14150257625641838) < 1e-13


@pytest.mark.slow
@pytest.mark.parametrize("N,P,unorm", [(19_200_000_000, 3, 1.526933573752539e-3),
                                       (32_000_000_000, 6, 1.2374127877503986e-3)])
def test_kron_oracle_published_large(N, P, unorm):
    un, _ = oracle.kron_norms(compute_mesh_size(N, P), P, 1)
    assert abs(un - unorm) < 1e-12 * unorm


@pytest.mark.parametrize("R", [2, 3, 4, 8])
def test_partition_invariance_threaded(R):
    """R in-process ranks (ThreadComm) reproduce the 1-rank golden norms and CSR."""
    nx = compute_mesh_size(1000 * R, 2) if R > 2 else (4, 3, 5)

    def body(comm):
        pb = _problem(nx, 2, 1, pert=0.1, comm=comm)
        u = pb.assemble_rhs()
        y = pb.new_vector()
        MatFreeLaplacianCPU(pb).apply(u, y)
        z = pb.new_vector()
        csr = CSROperator(pb)
        csr.apply(u, z)
        if comm.size > 1 and pb.halo.active and pb.halo.ghosts.total > 0:
            # the owned-column pass (run while the forward exchange is in
            # flight) never reads a ghost entry: poison them and check
            assert csr.nghost_entries > 0
            xp = u.clone()
            xp.view(-1)[pb.halo.ghosts.index] = float("nan")
            w = pb.new_vector()
            csr._spmv(csr.row_ptr[:-1], csr.off, xp, w, False)
            assert torch.isfinite(w).all()
        x = pb.new_vector()
        cg_solve(MatFreeLaplacianCPU(pb), pb, x, u, 5)
        return pb.norm(u), pb.norm(y), pb.norm(z - y), pb.norm(x)

    ref = body(Comm())
    for res in run_threaded(R, body):
        assert abs(res[0] - ref[0]) < 1e-12 * ref[0]
        assert abs(res[1] - ref[1]) < 1e-12 * ref[1]
        assert res[2] < 1e-12 * ref[1]
        assert abs(res[3] - ref[3]) < 1e-10 * ref[3]


@pytest.mark.parametrize("R", [1, 3])
def test_norms_and_blas1(R):
    def body(comm):
        pb = _problem((4, 3, 5), 2, 1, comm=comm)
        u = pb.assemble_rhs()
        v = pb.new_vector()
        pb.copy(v, u)
        pb.scale(v, -2.0)
        w = pb.new_vector()
        pb.axpy(w, 0.5, v, u)          # 0.5 * (-2u) + u = 0
        z = pb.new_vector()
        pb.pointwise_mult(z, u, u)
        return (pb.norm(u), pb.norm(v, "linf"), pb.norm(w), pb.inner(z, pb.new_vector() + 1.0),
                pb.norm(u) ** 2)

    res = run_threaded(R, body)
    ref = body(Comm())
    for r in res:
        assert abs(r[0] - ref[0]) < 1e-14 * ref[0]
        assert abs(r[1] - ref[1]) < 1e-14 * ref[1]   # linf = max |v| (not |max v|)
        assert r[2] < 1e-15
        assert abs(r[3] - r[4]) < 1e-12 * r[4]          # sum(u*u) == ||u||^2


@pytest.mark.parametrize("nc,P,qm,pert", [((3, 2, 4), 2, 1, 0.0), ((2, 3, 2), 3, 0, 0.2),
                                          ((2, 2, 2), 4, 1, 0.1)])
def test_random_coefficients_vs_oracle(nc, P, qm, pert):
    from benchmark_dolfinx_amd.fem.mesh import cell_coefficients
    pb = PoissonProblem(Comm(), nc, P, qm, False, torch.float64, "cpu", pert, "random")
    kc = cell_coefficients(make_local_lattice(0, 1, nc, P), "random")
    assert kc.shape == nc and kc.min() >= 1.0 and kc.max() < 3.0 and kc.std() > 0.1
    ref = oracle.box_model(nc, P, qm, vertices=_global_vertices(nc, pert), kappa_cells=kc)
    rng = np.random.default_rng(11)
    xg = rng.standard_normal(ref["u"].size)
    x = pb.new_vector()
    x[:, :, : pb.lat.L[2]] = torch.from_numpy(xg[pb.lat.global_indices()])
    y = pb.new_vector()
    MatFreeLaplacianCPU(pb).apply(x, y)
    yr = ref["apply"](xg)
    assert np.abs(pb.to_global_array(y) - yr).max() <= 1e-11 * np.abs(yr).max()
    z = pb.new_vector()
    CSROperator(pb).apply(x, z)
    assert np.abs(pb.to_global_array(z) - yr).max() <= 1e-11 * np.abs(yr).max()


@pytest.mark.parametrize("R", [2, 4])
def test_random_coefficients_partition_invariant(R):
    def body(comm):
        pb = _problem((5, 4, 6), 2, 1, pert=0.1, comm=comm)
        pb2 = PoissonProblem(comm, (5, 4, 6), 2, 1, False, torch.float64, "cpu", 0.1, "random")
        u = pb2.assemble_rhs()
        y = pb2.new_vector()
        MatFreeLaplacianCPU(pb2).apply(u, y)
        x = pb2.new_vector()
        cg_solve(MatFreeLaplacianCPU(pb2), pb2, x, u, 6)
        del pb
        return pb2.norm(y), pb2.norm(x)

    ref = body(Comm())
    for r in run_threaded(R, body):
        assert abs(r[0] - ref[0]) < 1e-12 * ref[0] and abs(r[1] - ref[1]) < 1e-10 * ref[1]
