"""Mesh sizing (reference src/mesh.cpp:117-152) and the analytic block
partition / halo tables (replaces ParMETIS + ghost_layer_mesh,
src/mesh.cpp:26-114): pure-function property tests simulating R ranks."""


import numpy as np
import pytest

from benchmark_dolfinx_amd.fem.mesh import (compute_mesh_size, make_local_lattice,
                                            partition_grid, vertex_coordinates)


@pytest.mark.parametrize("N,P,expect", [
    (1000, 3, (3, 3, 3)),
    (100000, 3, (12, 17, 17)),          # examples/mat_comp-16.json: 3468 cells
    (19_200_000_000, 3, (887, 893, 897)),  # examples/Q3-300M.json: 710505627 cells
    (32_000_000_000, 6, (524, 529, 534)),  # examples/Q6-500M.json: 148022664 cells
    (300_000_000, 3, (222, 223, 223)),
    (500_000_000, 6, (132, 132, 132)),
])
def test_compute_mesh_size(N, P, expect):
    assert compute_mesh_size(N, P) == expect


def test_published_cell_counts():
    assert np.prod(compute_mesh_size(19_200_000_000, 3)) == 710505627
    assert np.prod(compute_mesh_size(32_000_000_000, 6)) == 148022664
    nx = compute_mesh_size(19_200_000_000, 3)
    assert np.prod([n * 3 + 1 for n in nx]) == 19_205_158_720
    nx = compute_mesh_size(32_000_000_000, 6)
    assert np.prod([n * 6 + 1 for n in nx]) == 32_003_126_875


@pytest.mark.parametrize("R", [1, 2, 3, 4, 6, 8, 12, 16])
def test_partition_grid(R):
    p = partition_grid(R, (20, 21, 22))
    assert np.prod(p) == R


def test_partition_grid_8_is_cube():
    assert sorted(partition_grid(8, (100, 100, 100))) == [2, 2, 2]


CASES = [((3, 4, 5), 2, R) for R in (1, 2, 3, 4, 6, 8)] + [((5, 3, 4), 3, 4), ((4, 4, 4), 1, 8)]


@pytest.mark.parametrize("nc,P,R", CASES)
def test_partition_properties(nc, P, R):
    lats = [make_local_lattice(r, R, nc, P) for r in range(R)]
    N = lats[0].N
    owner = -np.ones(int(np.prod(N)), dtype=np.int64)
    ncells = 0
    for lat in lats:
        ncells += lat.ncells_local
        gi = lat.global_indices()
        oh = lat.owned_hi
        own = gi[: oh[0], : oh[1], : oh[2]].ravel()
        assert np.all(owner[own] == -1), "dof owned twice"
        owner[own] = lat.rank
        assert lat.ndofs_owned == own.size
    assert np.all(owner >= 0), "dof without owner"
    assert ncells == np.prod(nc)
    # every ghost plane dof is owned by the rank named in the recv boxes and
    # the recv/send boxes pair up exactly (same global dofs, same order)
    for lat in lats:
        gi = lat.global_indices()
        recv = lat.halo_recv_boxes()
        ghost = np.ones(lat.L, bool)
        oh = lat.owned_hi
        ghost[: oh[0], : oh[1], : oh[2]] = False
        covered = np.zeros(lat.L, bool)
        for hb in recv:
            sl = tuple(slice(l, h) for l, h in zip(hb.lo, hb.hi))
            assert not covered[sl].any()
            covered[sl] = True
            assert np.all(owner[gi[sl].ravel()] == hb.peer)
            peer = lats[hb.peer]
            sends = [s for s in peer.halo_send_boxes() if s.peer == lat.rank]
            assert len(sends) == 1
            s = sends[0]
            psl = tuple(slice(l, h) for l, h in zip(s.lo, s.hi))
            assert np.array_equal(peer.global_indices()[psl].ravel(), gi[sl].ravel())
        assert np.array_equal(covered, ghost)


@pytest.mark.parametrize("R", [1, 2, 4, 8])
def test_cell_boxes_cover_local_cells(R):
    for r in range(R):
        lat = make_local_lattice(r, R, (4, 5, 6), 2)
        m = np.zeros(lat.n, int)
        lo, hi = lat.interior_cell_box()
        m[tuple(slice(a, b) for a, b in zip(lo, hi))] += 1
        for lo, hi in lat.boundary_cell_boxes():
            m[tuple(slice(a, b) for a, b in zip(lo, hi))] += 1
        assert np.all(m == 1)
        # interior cells touch no ghost plane
        lo, hi = lat.interior_cell_box()
        for d in range(3):
            if lat.gh[d]:
                assert hi[d] * lat.degree < lat.L[d] - 1


def test_bc_mask_and_lattice():
    lat = make_local_lattice(0, 1, (2, 3, 4), 2)
    m = lat.bc_mask()
    assert m.shape == lat.L
    assert m.sum() == np.prod(lat.L) - np.prod([L - 2 for L in lat.L])
    assert lat.ld % 16 == 0 and lat.ld >= lat.L[2]
    d = lat.as_int64()
    assert d.dtype == np.int64 and d.size == 21


@pytest.mark.parametrize("R", [2, 4, 8])
def test_perturbation_partition_invariant(R):
    """Counter-based RNG keyed on the global vertex id (fixes quirk Q11)."""
    nc = (6, 5, 4)
    full = vertex_coordinates(make_local_lattice(0, 1, nc, 2), 0.2)
    for r in range(R):
        lat = make_local_lattice(r, R, nc, 2)
        X = vertex_coordinates(lat, 0.2)
        ref = full[lat.c0[0]: lat.c1[0] + 1, lat.c0[1]: lat.c1[1] + 1, lat.c0[2]: lat.c1[2] + 1]
        assert np.array_equal(X, ref)
    # only x moves, by at most 0.2/nx
    base = vertex_coordinates(make_local_lattice(0, 1, nc, 2), 0.0)
    dx = full - base
    assert np.all(dx[..., 1:] == 0) and np.abs(dx[..., 0]).max() <= 0.2 / nc[0]
    assert np.abs(dx[..., 0]).max() > 0


def test_parallelepiped_detection():
    from benchmark_dolfinx_amd.models.poisson import cells_all_parallelepipeds
    lat = make_local_lattice(0, 1, (4, 5, 3), 2)
    X = vertex_coordinates(lat, 0.0)
    assert cells_all_parallelepipeds(X)
    # a global affine map keeps every cell a parallelepiped (exact in binary
    # for these dyadic coefficients)
    A = np.array([[1.0, 0.5, 0.0], [0.0, 1.0, 0.25], [0.0, 0.0, 2.0]])
    Xa = (X * 8).round() / 8 @ A.T
    assert cells_all_parallelepipeds(Xa)
    assert not cells_all_parallelepipeds(vertex_coordinates(lat, 0.1))
    Xb = X.copy()
    Xb[2, 2, 1, 1] += 1e-9
    assert not cells_all_parallelepipeds(Xb)


def test_sheared_mesh_is_parallelepiped_with_full_jacobian():
    """The test-only shear map keeps every cell a parallelepiped (bitwise
    check) while making the Jacobian full, so the mixed geometry terms
    G01/G02/G12 are exercised (fused3's affine instance; fused5 refuses
    these cells)."""
    import torch
    from benchmark_dolfinx_amd.models.poisson import PoissonProblem
    from benchmark_dolfinx_amd.parallel.comm import Comm
    pb = PoissonProblem(Comm(), (4, 8, 8), 3, 1, False, torch.float64, "cpu", 0.0,
                        "constant", 0.5)
    assert pb.all_affine
    X = pb.xv_host
    J = np.stack([X[1, 0, 0] - X[0, 0, 0], X[0, 1, 0] - X[0, 0, 0], X[0, 0, 1] - X[0, 0, 0]], 1)
    off = J - np.diag(np.diag(J))
    assert np.all(np.abs(off[np.nonzero(off)]) > 0) and np.count_nonzero(off) == 3


def test_x_trilinear_classification():
    """The reference's --geom_perturb_fact moves vertex x only
    (src/mesh.cpp:199-207): such meshes are x-trilinear (fused3 AFF = 2);
    sheared meshes are not, boxes are."""
    import torch

    from benchmark_dolfinx_amd.models.poisson import PoissonProblem, cells_x_trilinear
    from benchmark_dolfinx_amd.parallel.comm import Comm
    box = PoissonProblem(Comm(), (3, 4, 5), 2, 1, False, torch.float64, "cpu")
    pert = PoissonProblem(Comm(), (3, 4, 5), 2, 1, False, torch.float64, "cpu", 0.2)
    shear = PoissonProblem(Comm(), (3, 4, 5), 2, 1, False, torch.float64, "cpu", 0.2,
                           "constant", 0.3)
    assert box.all_x_trilinear and box.all_affine
    assert pert.all_x_trilinear and not pert.all_affine
    assert not shear.all_x_trilinear
    X = pert.xv_host.copy()
    X[1, 2, 3, 1] += 1e-3  # one y coordinate off the lattice
    assert not cells_x_trilinear(X)
