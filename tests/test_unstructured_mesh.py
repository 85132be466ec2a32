"""The unstructured (dofmap) data model built from the box: every cell's dof
and vertex maps, the flags and the interior/boundary split agree with the
lattice, and renumbering is a consistent relabelling (CPU only; the GPU
operator on it is tested in test_gpu_dofmap.py)."""

import numpy as np
import pytest
import torch

from benchmark_dolfinx_amd.models.poisson import PoissonProblem
from benchmark_dolfinx_amd.models.unstructured import UnstructuredMesh
from benchmark_dolfinx_amd.parallel.comm import run_threaded


def _mesh(comm, nc, P, kappa="constant"):
    pb = PoissonProblem(comm, nc, P, 1, False, torch.float64, "cpu", 0.1, kappa)
    return pb, UnstructuredMesh.from_problem(pb)


@pytest.mark.parametrize("P", [1, 3, 6])
def test_dofmap_matches_lattice(P):
    pb, m = run_threaded(1, _mesh, (3, 4, 2), P)[0]
    lat = pb.lat
    nd = P + 1
    assert m.cell_dofs.shape == (lat.ncells_local, nd ** 3)
    assert m.ncells == lat.ncells_local and m.ndofs == lat.nstore
    # cell (cx, cy, cz) = row (cx n1 + cy) n2 + cz; dof (i, j, k) of that cell
    cx, cy, cz = 1, 2, 1
    row = (cx * lat.n[1] + cy) * lat.n[2] + cz
    for i, j, k in [(0, 0, 0), (P, 0, 1 % nd), (P, P, P)]:
        li, lj, lk = cx * P + i, cy * P + j, cz * P + k
        assert m.cell_dofs[row, (i * nd + j) * nd + k] == (li * lat.L[1] + lj) * lat.ld + lk
    # geometry nodes: vertex 7 of the cell is (cx+1, cy+1, cz+1)
    v7 = ((cx + 1) * (lat.n[1] + 1) + cy + 1) * (lat.n[2] + 1) + cz + 1
    assert m.cell_verts[row, 7] == v7
    assert np.array_equal(m.coords[v7], pb.xv_host.reshape(-1, 3)[v7])
    # every referenced dof is a real lattice point; flags = bc | owned << 1
    flags = m.dof_flags.reshape(lat.shape)[:, :, :lat.L[2]]
    assert np.array_equal(flags & 1, lat.bc_mask().astype(np.uint8))
    assert np.array_equal(flags >> 1, lat.owned_mask().astype(np.uint8))
    assert len(m.interior_cells) == lat.ncells_local and len(m.boundary_cells) == 0


def test_interior_boundary_split_on_ranks():
    res = run_threaded(4, _mesh, (4, 6, 6), 2)
    for pb, m in res:
        lat = pb.lat
        both = np.concatenate([m.interior_cells, m.boundary_cells])
        assert np.array_equal(np.sort(both), np.arange(m.ncells))
        hi = [n - g for n, g in zip(lat.n, lat.gh)]
        assert len(m.interior_cells) == int(np.prod(hi))
        # a boundary cell touches a ghost dof (a non-owned flag)
        owned = (m.dof_flags >> 1) & 1
        for c in m.boundary_cells[:20]:
            assert not owned[m.cell_dofs[c]].all()
        for c in m.interior_cells[:20]:
            assert owned[m.cell_dofs[c]].all()


def test_renumbering_is_a_relabelling():
    pb, m = run_threaded(1, _mesh, (2, 3, 2), 3, "random")[0]
    rng = np.random.default_rng(5)
    dp = rng.permutation(m.ndofs)
    cp = rng.permutation(m.ncells)
    vp = rng.permutation(m.coords.shape[0])
    r = m.renumbered(dp, cp, vp)
    # row pos of r is cell cp[pos] of m
    assert np.array_equal(r.cell_dofs, dp[m.cell_dofs[cp]])
    assert np.array_equal(r.coords[r.cell_verts], m.coords[m.cell_verts[cp]])
    assert np.array_equal(r.dof_flags[dp], m.dof_flags)
    assert np.array_equal(r.kc, m.kc[cp])
    assert sorted(cp[r.interior_cells].tolist()) == sorted(m.interior_cells.tolist())
