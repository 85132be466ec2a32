"""Box mesh sizing and the analytic block partition.

The reference builds a distributed hexahedral box mesh with DOLFINx/ParMETIS
(`src/mesh.cpp:190-218`) and re-creates it with a one-cell ghost layer
(`src/mesh.cpp:26-114`).  Here the mesh is a structured lattice by
construction, so the partition, the dof numbering and the halo pattern are
all analytic:

* the global box of ``n = (nx, ny, nz)`` cells is split into
  ``px x py x pz`` blocks of cells (one block per rank, surface-minimising
  factorisation, `partition_grid`);
* rank r owns the cells ``[c0, c1)`` in each axis; its local dof lattice is
  ``[c0*P, c1*P]`` (inclusive) per axis, stored lexicographically with z
  fastest;
* the upper plane ``c1*P`` of an axis is a *ghost* plane when an upper
  neighbour exists in that axis (it is owned by that neighbour), otherwise
  it is the global boundary and owned;
* there are no ghost cells: each cell is computed by exactly one rank, so an
  operator apply needs one forward halo exchange (owner -> ghost plane
  values of the input) and one reverse exchange (ghost-plane partial sums ->
  owner).  Both are plane-sized (1 dof thick), which is P times less data per
  exchange than the reference's one-cell ghost layer.
"""

from __future__ import annotations

import itertools
import math
from dataclasses import dataclass, field

import numpy as np


def compute_mesh_size(ndofs_global: int, degree: int) -> tuple[int, int, int]:
    """Choose (nx, ny, nz) so that prod(n_d*P+1) is closest to ndofs_global.

    Same search as the reference (`src/mesh.cpp:117-152`): seed
    n0 = round((N^(1/3) - 1) / P), then scan n0-5..n0+5 in each axis (x outer,
    z inner) keeping the first strict improvement.
    """
    P = int(degree)
    N = int(ndofs_global)
    nx_approx = (N ** (1.0 / 3.0) - 1.0) / P
    n0 = int(nx_approx + 0.5)
    best = abs((n0 * P + 1) ** 3 - N)
    nx = (n0, n0, n0)
    lo = max(1, n0 - 5)
    for a in range(lo, n0 + 6):
        fa = a * P + 1
        for b in range(lo, n0 + 6):
            fb = fa * (b * P + 1)
            for c in range(lo, n0 + 6):
                misfit = abs(fb * (c * P + 1) - N)
                if misfit < best:
                    best = misfit
                    nx = (a, b, c)
    return nx


def partition_grid(nranks: int, ncells: tuple[int, int, int],
                   whole_x: bool = False) -> tuple[int, int, int]:
    """Factor nranks into (px, py, pz) minimising the cut area.

    Cut area = sum_d (p_d - 1) * (cross-section normal to d).  Ties prefer
    splitting x first (x-planes are contiguous in the z-fastest layout).

    ``whole_x``: never split x (px = 1) when a (y, z) split exists.  The fused
    GPU kernels march along x over (y, z) tiles; with x whole only the last
    tile row / column touches a ghost plane, so the native runtime runs every
    other tile while the halo exchange is in flight (csrc/hip/runtime.hip).
    That costs some cut area (8 ranks on a cube: 1x2x4, +32 %) for halos that
    are hidden instead of exposed.
    """
    if whole_x:
        try:
            return partition_grid(nranks, (1, ncells[1], ncells[2]))
        except ValueError:
            pass
    nx, ny, nz = ncells
    best = None
    for px in range(1, nranks + 1):
        if nranks % px:
            continue
        for py in range(1, nranks // px + 1):
            if (nranks // px) % py:
                continue
            pz = nranks // (px * py)
            if px > nx or py > ny or pz > nz:
                continue
            cost = (px - 1) * ny * nz + (py - 1) * nx * nz + (pz - 1) * nx * ny
            key = (cost, -px, -py)
            if best is None or key < best[0]:
                best = (key, (px, py, pz))
    if best is None:
        raise ValueError(f"Cannot partition {ncells} cells over {nranks} ranks")
    return best[1]


@dataclass
class HaloBox:
    """A box of local lattice indices exchanged with one peer."""

    peer: int
    lo: tuple[int, int, int]
    hi: tuple[int, int, int]  # exclusive

    @property
    def size(self) -> int:
        return int(np.prod([h - l for l, h in zip(self.lo, self.hi)]))


@dataclass
class LocalLattice:
    """Everything one rank needs to know about its piece of the box.

    Index conventions: axis 0 = x (slowest), axis 2 = z (fastest).
    """

    rank: int
    nranks: int
    degree: int
    ncells_global: tuple[int, int, int]
    pgrid: tuple[int, int, int]
    rcoord: tuple[int, int, int]
    c0: tuple[int, int, int]
    c1: tuple[int, int, int]
    # derived
    n: tuple[int, int, int] = field(init=False)
    L: tuple[int, int, int] = field(init=False)
    g0: tuple[int, int, int] = field(init=False)
    N: tuple[int, int, int] = field(init=False)
    gh: tuple[int, int, int] = field(init=False)

    def __post_init__(self):
        P = self.degree
        self.n = tuple(int(b - a) for a, b in zip(self.c0, self.c1))
        self.L = tuple(int(m * P + 1) for m in self.n)
        self.g0 = tuple(int(a * P) for a in self.c0)
        self.N = tuple(int(m * P + 1) for m in self.ncells_global)
        self.gh = tuple(int(r < p - 1) for r, p in zip(self.rcoord, self.pgrid))

    # ---------------------------------------------------------------- sizes
    @property
    def ndofs_local(self) -> int:
        """Local lattice size (owned + ghost planes)."""
        return int(np.prod(self.L))

    @property
    def owned_hi(self) -> tuple[int, int, int]:
        return tuple(L - g for L, g in zip(self.L, self.gh))

    @property
    def ndofs_owned(self) -> int:
        return int(np.prod(self.owned_hi))

    @property
    def ncells_local(self) -> int:
        return int(np.prod(self.n))

    @property
    def ndofs_global(self) -> int:
        return int(np.prod(self.N))

    @property
    def ncells_global_total(self) -> int:
        return int(np.prod(self.ncells_global))

    @property
    def ld(self) -> int:
        """z pitch of the storage: rows padded to a multiple of 16 elements."""
        return int(-(-self.L[2] // 16) * 16)

    @property
    def shape(self) -> tuple[int, int, int]:
        """Storage shape of a local vector (padded z pitch)."""
        return (self.L[0], self.L[1], self.ld)

    @property
    def nstore(self) -> int:
        return self.L[0] * self.L[1] * self.ld

    def as_int64(self, tile: tuple[int, int] | None = None) -> np.ndarray:
        """Packed descriptor passed to native code (layout: csrc/include/bdx_lattice.h).
        `tile` = (tsy, tsz) node sizes selects the tiled storage layout."""
        tl = [0, 0, 0, 0]
        if tile is not None:
            tsy, tsz = tile
            tl = [tsy, tsz, (self.L[2] - 1) // tsz + 1, self.L[0] * tsy * tsz]
        return np.array(list(self.n) + list(self.L) + list(self.g0) + list(self.N)
                        + list(self.gh) + [self.degree, self.ld] + tl, dtype=np.int64)

    def tiled_size(self, tsy: int, tsz: int) -> int:
        """Elements of a vector in the tiled storage layout (tiles of tsy x tsz
        nodes, each tile's x-column contiguous; bdx_lattice.h)."""
        return ((self.L[1] - 1) // tsy + 1) * ((self.L[2] - 1) // tsz + 1) * self.L[0] * tsy * tsz

    # ------------------------------------------------------------- topology
    def rank_of(self, coord) -> int:
        px, py, pz = self.pgrid
        return (coord[0] * py + coord[1]) * pz + coord[2]

    def interior_cell_box(self):
        """Cells that touch no ghost dof (computable before the halo arrives)."""
        return (0, 0, 0), tuple(m - g for m, g in zip(self.n, self.gh))

    def boundary_cell_boxes(self):
        """Disjoint boxes covering the cells that touch a ghost plane."""
        boxes = []
        hi = list(self.n)
        for d in range(3):
            if self.gh[d] and self.n[d] > 0:
                lo = [0, 0, 0]
                bh = list(hi)
                lo[d] = self.n[d] - 1
                bh[d] = self.n[d]
                boxes.append((tuple(lo), tuple(bh)))
                hi[d] = self.n[d] - 1
        return [b for b in boxes if all(h > l for l, h in zip(*b))]

    def halo_recv_boxes(self) -> list[HaloBox]:
        """Ghost blocks (forward: received from upper neighbours)."""
        out = []
        for S in itertools.product((0, 1), repeat=3):
            if not any(S):
                continue
            if any(s and not g for s, g in zip(S, self.gh)):
                continue
            lo, hi = [], []
            for d in range(3):
                if S[d]:
                    lo.append(self.L[d] - 1)
                    hi.append(self.L[d])
                else:
                    lo.append(0)
                    hi.append(self.L[d] - self.gh[d])
            peer = self.rank_of(tuple(r + s for r, s in zip(self.rcoord, S)))
            out.append(HaloBox(peer, tuple(lo), tuple(hi)))
        return out

    def halo_send_boxes(self) -> list[HaloBox]:
        """Owned lower-face blocks (forward: sent to lower neighbours)."""
        out = []
        for S in itertools.product((0, 1), repeat=3):
            if not any(S):
                continue
            if any(s and r == 0 for s, r in zip(S, self.rcoord)):
                continue
            lo, hi = [], []
            for d in range(3):
                if S[d]:
                    lo.append(0)
                    hi.append(1)
                else:
                    lo.append(0)
                    hi.append(self.L[d] - self.gh[d])
            peer = self.rank_of(tuple(r - s for r, s in zip(self.rcoord, S)))
            out.append(HaloBox(peer, tuple(lo), tuple(hi)))
        return out

    def owned_mask(self) -> np.ndarray:
        m = np.zeros(self.L, dtype=bool)
        oh = self.owned_hi
        m[:oh[0], :oh[1], :oh[2]] = True
        return m

    def global_indices(self) -> np.ndarray:
        """Global lexicographic dof index of every local lattice point."""
        ix = np.arange(self.L[0]) + self.g0[0]
        iy = np.arange(self.L[1]) + self.g0[1]
        iz = np.arange(self.L[2]) + self.g0[2]
        return ((ix[:, None, None] * self.N[1] + iy[None, :, None]) * self.N[2]
                + iz[None, None, :])

    def bc_mask(self) -> np.ndarray:
        """Dirichlet dofs (global boundary of the unit cube) in the local lattice."""
        m = np.zeros(self.L, dtype=bool)
        for d in range(3):
            g = np.arange(self.L[d]) + self.g0[d]
            on = (g == 0) | (g == self.N[d] - 1)
            shape = [1, 1, 1]
            shape[d] = self.L[d]
            m |= on.reshape(shape)
        return m


def make_local_lattice(rank: int, nranks: int, ncells: tuple[int, int, int],
                       degree: int, whole_x: bool = False) -> LocalLattice:
    pgrid = partition_grid(nranks, ncells, whole_x)
    px, py, pz = pgrid
    rz = rank % pz
    ry = (rank // pz) % py
    rx = rank // (py * pz)
    rc = (rx, ry, rz)
    c0 = tuple((ncells[d] * rc[d]) // pgrid[d] for d in range(3))
    c1 = tuple((ncells[d] * (rc[d] + 1)) // pgrid[d] for d in range(3))
    return LocalLattice(rank, nranks, degree, tuple(ncells), pgrid, rc, c0, c1)


def vertex_coordinates(lat: LocalLattice, perturb: float = 0.0,
                       seed: int = 42, shear: float = 0.0) -> np.ndarray:
    """Local vertex lattice coordinates, shape (nx+1, ny+1, nz+1, 3).

    With ``perturb != 0`` the x coordinate of every vertex (boundary vertices
    included, like `src/mesh.cpp:199-207`) moves by U(-perturb/nx, perturb/nx).
    The random value is a counter-based hash of the *global* vertex id, so the
    mesh is identical for every partition (fixes reference quirk Q11).

    ``shear != 0`` applies the global linear map (x, y, z) -> (x + s y,
    y + s z, z + s x): every cell stays a parallelepiped but its Jacobian is
    full (all geometry factors nonzero).  Test-only; with power-of-two cell
    counts and a dyadic s the map is exact in floating point, so the
    bitwise parallelepiped check still holds.
    """
    nxg, nyg, nzg = lat.ncells_global
    vx = np.arange(lat.c0[0], lat.c1[0] + 1, dtype=np.float64)
    vy = np.arange(lat.c0[1], lat.c1[1] + 1, dtype=np.float64)
    vz = np.arange(lat.c0[2], lat.c1[2] + 1, dtype=np.float64)
    X = np.empty((vx.size, vy.size, vz.size, 3), dtype=np.float64)
    X[..., 0] = (vx / nxg)[:, None, None]
    X[..., 1] = (vy / nyg)[None, :, None]
    X[..., 2] = (vz / nzg)[None, None, :]
    if perturb != 0.0:
        gid = ((np.arange(lat.c0[0], lat.c1[0] + 1, dtype=np.uint64)[:, None, None]
                * np.uint64(nyg + 1)
                + np.arange(lat.c0[1], lat.c1[1] + 1, dtype=np.uint64)[None, :, None])
               * np.uint64(nzg + 1)
               + np.arange(lat.c0[2], lat.c1[2] + 1, dtype=np.uint64)[None, None, :])
        u = _hash_uniform(gid, seed)
        amp = perturb / nxg
        X[..., 0] += (2.0 * u - 1.0) * amp
    if shear != 0.0:
        x0, y0, z0 = X[..., 0].copy(), X[..., 1].copy(), X[..., 2].copy()
        X[..., 0] = x0 + shear * y0
        X[..., 1] = y0 + shear * z0
        X[..., 2] = z0 + shear * x0
    return X


def _hash_uniform(ids: np.ndarray, seed: int) -> np.ndarray:
    """splitmix64 of (id, seed) -> uniform [0, 1)."""
    with np.errstate(over="ignore"):
        z = ids.astype(np.uint64) + np.uint64((seed * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF)
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def cells_per_dof_estimate(degree: int) -> float:
    return 1.0 / math.pow(degree, 3)


def cell_coefficients(lat: LocalLattice, mode: str = "constant", kappa: float = 2.0,
                      seed: int = 7):
    """Per-cell diffusion coefficient of the local cells, shape (n0, n1, n2), or
    None for the reference's constant kappa (src/main.cpp:71; the reference
    stores it per cell, src/laplacian.hpp:105).  mode="random": kappa_c =
    U(1, 3) from a counter-based hash of the *global* cell id, so every
    partition sees the same field."""
    if mode == "constant":
        return None
    if mode != "random":
        raise ValueError(f"unknown coefficient mode {mode}")
    nxg, nyg, nzg = lat.ncells_global
    gid = ((np.arange(lat.c0[0], lat.c1[0], dtype=np.uint64)[:, None, None] * np.uint64(nyg)
            + np.arange(lat.c0[1], lat.c1[1], dtype=np.uint64)[None, :, None]) * np.uint64(nzg)
           + np.arange(lat.c0[2], lat.c1[2], dtype=np.uint64)[None, None, :])
    return 1.0 + 2.0 * _hash_uniform(gid, seed)
