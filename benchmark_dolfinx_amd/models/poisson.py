"""The benchmark problem: -div(kappa grad u) = f on the unit cube, Q_P hexes.

Reference: `run_benchmark<T>` (src/main.cpp:41-133) and the operator classes
MatFreeLaplacianGPU/CPU (src/laplacian.hpp:87-771) and MatrixOperator
(src/csr.hpp:113-234).

* `PoissonProblem` builds the rank-local lattice, the 1D tables, the mesh
  vertices (optionally perturbed), interpolates f and assembles the RHS
  b = M f with Dirichlet rows zeroed (src/laplacian_solver.cpp:100-105).
* `MatFreeLaplacianCPU` / `MatFreeLaplacianGPU` apply y = A u with the
  reference's BC semantics (A = kappa K with Dirichlet rows/columns replaced
  by the identity).  One forward halo exchange of u overlapped with the
  interior cells, one reverse exchange of the ghost-plane partial sums.
* `CSROperator` is the assembled-matrix comparison operator (--mat_comp).
"""

from __future__ import annotations

import math
import os

import numpy as np
import torch

from ..fem.mesh import (LocalLattice, cell_coefficients, make_local_lattice,
                        vertex_coordinates)
from ..fem.quadrature import OperatorTables
from ..ops import native
from ..ops.native import ptr
from ..parallel.comm import Comm
from ..parallel.halo import HaloExchange
from ..utils.timing import timed

KAPPA = 2.0  # src/main.cpp:71


def _np_dtype(dtype):
    return np.float64 if dtype == torch.float64 else np.float32


def cells_axis_aligned(X: np.ndarray) -> bool:
    """True iff every cell edge of the vertex lattice X (nx+1, ny+1, nz+1, 3)
    along lattice axis a has exactly zero components along the other axes:
    the cells are boxes with diagonal Jacobians, so the geometry factors
    G01 = G02 = G12 vanish exactly (the fused5 2-array kernel instance)."""
    for ax in range(3):
        E = np.diff(X, axis=ax)
        for d in range(3):
            if d != ax and E[..., d].size and np.any(E[..., d] != 0):
                return False
    return True


def cells_x_trilinear(X: np.ndarray) -> bool:
    """True iff the vertex y coordinates of the lattice X (nx+1, ny+1, nz+1, 3)
    depend on the y index only and the z coordinates on the z index only
    (bitwise), so every cell's Jacobian is [[x_s, x_t, x_u], [0, hy, 0],
    [0, 0, hz]]: the class of `src/mesh.cpp:199-207`'s x-only perturbation.
    Selects fused3's x-trilinear instance (AFF = 2)."""
    for d, axes in ((1, (0, 2)), (2, (0, 1))):
        for ax in axes:
            E = np.diff(X[..., d], axis=ax)
            if E.size and np.any(E != 0):
                return False
    return True


def cells_all_parallelepipeds(X: np.ndarray) -> bool:
    """True iff every cell of the vertex lattice X (nx+1, ny+1, nz+1, 3) has
    bitwise-equal parallel edges (constant Jacobian).  Evaluated in the
    kernel's precision (X's dtype), so the kernel's affine path sees exactly
    the edge vectors checked here."""
    if X.shape[0] < 2 or X.shape[1] < 2 or X.shape[2] < 2:
        return True
    for ax in range(3):
        E = np.diff(X, axis=ax)
        others = [d for d in range(3) if d != ax]
        for d in others:
            sl_a = [slice(None)] * 4
            sl_b = [slice(None)] * 4
            sl_a[d] = slice(0, -1)
            sl_b[d] = slice(1, None)
            if not np.array_equal(E[tuple(sl_a)], E[tuple(sl_b)]):
                return False
    return True


class PoissonProblem:
    def __init__(self, comm: Comm, ncells, degree: int, qmode: int = 1,
                 use_gauss: bool = False, dtype=torch.float64, platform: str = "gpu",
                 perturb: float = 0.0, coefficient: str = "constant", shear: float = 0.0,
                 partition: str | None = None):
        if use_gauss and qmode == 0:
            # same validation as the reference (src/laplacian.hpp:197-198, Q5)
            raise RuntimeError("Expecting identity matrix for qmode=0")
        self.comm = comm
        self.platform = platform
        self.device = torch.device("cuda", torch.cuda.current_device()) \
            if platform == "gpu" else torch.device("cpu")
        self.dtype = dtype
        self.kappa = KAPPA
        self.degree = degree
        self.qmode = qmode
        self.use_gauss = use_gauss
        self.tables = OperatorTables(degree, qmode, use_gauss)
        # "yz": keep the march axis x whole (halo/compute overlap of the fused
        # GPU runtime); "xyz": minimum cut area.  Default: yz on the GPU.
        partition = partition or os.environ.get("BDX_PARTITION") or (
            "yz" if platform == "gpu" else "xyz")
        if partition not in ("yz", "xyz"):
            raise ValueError(f"unknown partition policy {partition!r}")
        self.partition = partition
        self.lat: LocalLattice = make_local_lattice(comm.rank, comm.size, tuple(ncells), degree,
                                                    whole_x=partition == "yz")
        npdt = _np_dtype(dtype)
        with timed("~setup mesh"):
            xv = vertex_coordinates(self.lat, perturb, shear=shear).astype(npdt)
            self.xv_host = np.ascontiguousarray(xv)
            self.xv = torch.from_numpy(self.xv_host).to(self.device)
        self.host_tables = {k: np.ascontiguousarray(v, dtype=npdt) for k, v in dict(
            phi0=self.tables.phi0, dphi1=self.tables.dphi1, wts=self.tables.qwts,
            qpts=self.tables.qpts, nodes=self.tables.nodes, B=self.tables.B,
            Dd=self.tables.Dd).items()}
        self.kernels = None
        if platform == "gpu":
            from ..ops.kernels import HipKernels
            self.kernels = HipKernels(self.lat, self.tables, dtype)
        self.halo = HaloExchange(self.lat, comm, dtype, self.device, self.kernels)
        # kept alive for ctypes calls (never pass temporaries to ptr())
        self.latd = self.lat.as_int64()
        self.all_affine = cells_all_parallelepipeds(self.xv_host)
        self.all_axis_aligned = self.all_affine and cells_axis_aligned(self.xv_host)
        self.all_x_trilinear = cells_x_trilinear(self.xv_host)
        # per-cell kappa (None: the reference's constant kappa = 2)
        self.coefficient = coefficient
        kc = cell_coefficients(self.lat, coefficient, KAPPA)
        self.kc_host = None if kc is None else np.ascontiguousarray(kc, dtype=npdt)
        self.kc = None if kc is None else torch.from_numpy(self.kc_host).to(self.device)

    # --------------------------------------------------------------- vectors
    @property
    def suf(self) -> str:
        return "f64" if self.dtype == torch.float64 else "f32"

    def new_vector(self) -> torch.Tensor:
        return torch.zeros(self.lat.shape, dtype=self.dtype, device=self.device)

    def owned(self, v: torch.Tensor) -> torch.Tensor:
        o = self.lat.owned_hi
        return v[: o[0], : o[1], : o[2]]

    def inner(self, a: torch.Tensor, b: torch.Tensor) -> float:
        s = torch.sum(self.owned(a).double() * self.owned(b).double())
        if self.comm.size > 1:
            self.comm.allreduce_(s.view(1) if s.dim() == 0 else s)
        return float(s.item())

    def norm(self, v: torch.Tensor, kind: str = "l2") -> float:
        """l2 or linf norm over the owned dofs (reference la::norm,
        src/vector.hpp:196-218; linf here is max |v|, not the reference's
        |max v| (quirk Q7))."""
        if kind == "l2":
            return math.sqrt(max(self.inner(v, v), 0.0))
        if kind != "linf":
            raise ValueError(f"unknown norm {kind}")
        m = torch.max(torch.abs(self.owned(v))).double().reshape(1)
        if self.comm.size > 1:
            m = m.to(self.comm.device)
            self.comm.allreduce_(m, "max")
        return float(m.item())

    # BLAS-1 over the owned dofs (reference src/vector.hpp:228-292: axpy,
    # scale, copy, pointwise_mult, set_value); vectors keep the padded layout
    def axpy(self, out: torch.Tensor, alpha: float, x: torch.Tensor, y: torch.Tensor) -> None:
        self.owned(out).copy_(alpha * self.owned(x) + self.owned(y))

    def scale(self, v: torch.Tensor, alpha: float) -> None:
        self.owned(v).mul_(alpha)

    def copy(self, dst: torch.Tensor, src: torch.Tensor) -> None:
        self.owned(dst).copy_(self.owned(src))

    def pointwise_mult(self, out: torch.Tensor, x: torch.Tensor, y: torch.Tensor) -> None:
        self.owned(out).copy_(self.owned(x) * self.owned(y))

    def set_value(self, v: torch.Tensor, value: float) -> None:
        v.fill_(value)  # owned + ghost, like the reference

    def bc_mask(self) -> torch.Tensor:
        m = np.zeros(self.lat.shape, dtype=bool)
        m[:, :, : self.lat.L[2]] = self.lat.bc_mask()
        return torch.from_numpy(m).to(self.device)

    def to_global_array(self, v: torch.Tensor) -> np.ndarray:
        """Gather the owned values into a global lexicographic numpy array (tests)."""
        o = self.lat.owned_hi
        loc = self.owned(v).detach().cpu().numpy().astype(np.float64)
        gidx = self.lat.global_indices()[: o[0], : o[1], : o[2]]
        parts = self.comm.gather_objects((gidx.ravel(), loc.ravel()))
        out = np.zeros(self.lat.ndofs_global)
        for gi, val in parts:
            out[gi] = val
        return out

    # -------------------------------------------------------------- RHS
    def interpolate_f(self) -> torch.Tensor:
        """f at the physical dof nodes (src/main.cpp:81-92), all local points."""
        f = np.zeros(self.lat.shape, dtype=_np_dtype(self.dtype))
        lib = native.host()
        getattr(lib, f"bdx_cpu_interp_f_{self.suf}")(
            ptr(self.latd), ptr(self.host_tables["nodes"]), ptr(self.xv_host), ptr(f))
        return torch.from_numpy(f).to(self.device)

    def assemble_rhs(self) -> torch.Tensor:
        """b = M f, reverse-scattered, Dirichlet rows zeroed."""
        with timed("~setup assemble RHS"):
            f = self.interpolate_f()
            b = self.new_vector()
            lo = np.zeros(3, dtype=np.int64)
            hi = np.array(self.lat.n, dtype=np.int64)
            if self.platform == "gpu":
                self.kernels.v1_apply(2, None, self.xv, 0.0, f, b, lo, hi)
            else:
                t = self.host_tables
                getattr(native.host(), f"bdx_cpu_mass_{self.suf}")(
                    ptr(self.latd), self.tables.nq, ptr(t["phi0"]), ptr(t["dphi1"]),
                    ptr(t["wts"]), ptr(t["qpts"]), ptr(t["nodes"]), int(self.tables.is_identity),
                    ptr(self.xv_host), ptr(f.numpy()), ptr(b.numpy()), ptr(lo), ptr(hi))
            self.halo.reverse(b)
            b.masked_fill_(self.bc_mask(), 0.0)
            self.halo.forward(b)
        return b

    @property
    def ndofs_global(self) -> int:
        return self.lat.ndofs_global

    @property
    def ncells_global(self) -> int:
        return self.lat.ncells_global_total


class MatFreeLaplacianCPU:
    """CPU operator (C++/OpenMP, both qmodes; src/laplacian.hpp:450-771)."""

    # geometry factors precomputed per cell (reference layout [c][6][nq^3],
    # src/laplacian.hpp:515-541) when they fit in this many bytes, else
    # computed per point on the fly.  Default 0 (on the fly): on this 8-core
    # host the stored-G apply is memory-bound and slower at 8 threads (73 vs
    # 49 ms per 1 M DoF Q3 apply; faster on one thread, 182 vs 365 ms).
    # BDX_CPU_G_MAX_BYTES overrides.
    G_MAX_BYTES = 0

    def __init__(self, problem: PoissonProblem):
        import os
        self.pb = problem
        self.lib = native.host()
        self._fn = getattr(self.lib, f"bdx_cpu_stiffness_g_{problem.suf}")
        self.latd = problem.lat.as_int64()
        nq = problem.tables.nq
        ncells = int(np.prod(problem.lat.n))
        nbytes = ncells * 6 * nq ** 3 * problem.new_vector().element_size()
        self.G = None
        if nbytes <= int(os.environ.get("BDX_CPU_G_MAX_BYTES", self.G_MAX_BYTES)):
            t = problem.host_tables
            self.G = np.empty(ncells * 6 * nq ** 3, dtype=t["wts"].dtype)
            getattr(self.lib, f"bdx_cpu_geometry_{problem.suf}")(
                ptr(self.latd), nq, ptr(t["wts"]), ptr(t["qpts"]), ptr(problem.xv_host),
                ptr(self.G))

    def _cells(self, u, y, lo, hi):
        t = self.pb.host_tables
        lo = np.asarray(lo, dtype=np.int64)
        hi = np.asarray(hi, dtype=np.int64)
        self._fn(ptr(self.latd), self.pb.tables.nq, ptr(t["phi0"]), ptr(t["dphi1"]),
                 ptr(t["wts"]), ptr(t["qpts"]), ptr(t["nodes"]),
                 int(self.pb.tables.is_identity), ptr(self.pb.xv_host),
                 ptr(self.G) if self.G is not None else None, self.pb.kappa,
                 ptr(self.pb.kc_host), ptr(u.numpy()), ptr(y.numpy()), ptr(lo), ptr(hi))

    def apply(self, u: torch.Tensor, y: torch.Tensor) -> None:
        lat = self.pb.lat
        y.zero_()
        work = self.pb.halo.forward_begin(u)
        lo, hi = lat.interior_cell_box()
        self._cells(u, y, lo, hi)
        self.pb.halo.forward_end(u, work)
        for lo, hi in lat.boundary_cell_boxes():
            self._cells(u, y, lo, hi)
        self.pb.halo.reverse(y)


class MatFreeLaplacianGPU:
    """Matrix-free operator on the GPU.

    geometry="stored": G precomputed once (6 nq^3 values per cell, the
    reference's memory layout and maths); "otf": G recomputed per
    quadrature point from the 8 vertices of the cell (no G array).
    """

    def __init__(self, problem: PoissonProblem, geometry: str = "stored"):
        self.pb = problem
        self.k = problem.kernels
        self.geometry = geometry
        self.G = None
        if geometry == "stored":
            lat = problem.lat
            nq3 = problem.tables.nq ** 3
            with timed("~setup geometry"):
                self.G = torch.empty(lat.ncells_local * 6 * nq3, dtype=problem.dtype,
                                     device=problem.device)
                self.k.geometry(problem.xv, self.G)
        elif geometry != "otf":
            raise ValueError(f"unknown geometry mode {geometry}")
        self.mode = 0 if geometry == "stored" else 1

    def apply(self, u: torch.Tensor, y: torch.Tensor) -> None:
        pb, lat = self.pb, self.pb.lat
        y.zero_()
        work = pb.halo.forward_begin(u)
        lo, hi = lat.interior_cell_box()
        self.k.v1_apply(self.mode, self.G, pb.xv, pb.kappa, u, y, lo, hi, pb.kc)
        pb.halo.forward_end(u, work)
        for lo, hi in lat.boundary_cell_boxes():
            self.k.v1_apply(self.mode, self.G, pb.xv, pb.kappa, u, y, lo, hi, pb.kc)
        pb.halo.reverse(y)


class CSROperator:
    """Assembled local stiffness matrix (rows = local lattice incl. ghost rows).

    Assembly on the CPU (C++), SpMV on the device of the problem; the ghost
    rows' partial sums go through the same reverse halo exchange as the
    matrix-free operator (the reference assembles owned rows via
    MatrixCSR::scatter_rev, src/laplacian_solver.cpp:183).
    """

    def __init__(self, problem: PoissonProblem):
        self.pb = problem
        lat = problem.lat
        if lat.nstore >= 2 ** 31:
            raise RuntimeError("Too many matrix rows for int32 columns")
        lib = native.host()
        fn = getattr(lib, f"bdx_cpu_csr_{problem.suf}")
        t = problem.host_tables
        npdt = _np_dtype(problem.dtype)
        row_ptr = np.zeros(lat.nstore + 1, dtype=np.int64)
        self.latd = problem.latd
        args = (ptr(self.latd), problem.tables.nq, ptr(t["B"]), ptr(t["Dd"]),
                ptr(t["wts"]), ptr(t["qpts"]), ptr(problem.xv_host), problem.kappa,
                ptr(problem.kc_host))
        with timed("% Create CPU MatrixCSR"):
            nnz = fn(*args, ptr(row_ptr), 0, 0, 1)
            if nnz >= 2 ** 31:
                raise RuntimeError("Too many matrix entries, need 64-bit row_ptr.")
            cols = np.zeros(nnz, dtype=np.int32)
            vals = np.zeros(nnz, dtype=npdt)
            row_ptr[:] = 0
        with timed("% Assemble CPU MatrixCSR"):
            fn(*args, ptr(row_ptr), ptr(cols), ptr(vals), 0)
        self.nnz = int(nnz)
        self.nrows = lat.nstore
        # Column split of every row, as DOLFINx's MatrixCSR off-diagonal block
        # (src/csr.hpp:203-217): entries [row_ptr, off) read columns this rank
        # owns or computes itself, [off, row_ptr + 1) the ghost columns that the
        # forward halo exchange fills -- so the first pass overlaps it.
        ghost = np.zeros(lat.nstore, dtype=bool)
        halo = problem.halo
        if getattr(halo, "active", False):
            ghost[halo.ghosts.index.cpu().numpy()] = True
        rows = np.repeat(np.arange(lat.nstore, dtype=np.int64), np.diff(row_ptr))
        g = ghost[cols]
        order = np.lexsort((g, rows))  # stable: by row, owned columns first
        cols, vals = np.ascontiguousarray(cols[order]), np.ascontiguousarray(vals[order])
        off = row_ptr[:-1] + np.bincount(rows[~g], minlength=lat.nstore).astype(np.int64)
        self.nghost_entries = int(g.sum())
        with timed("% Copy to GPU MatrixCSR" if problem.platform == "gpu"
                   else "% Copy CSR"):
            dev = problem.device
            self.row_ptr = torch.from_numpy(row_ptr).to(dev)
            self.off = torch.from_numpy(off).to(dev)
            self.cols = torch.from_numpy(cols).to(dev)
            self.vals = torch.from_numpy(vals).to(dev)
        self._host = (row_ptr, cols, vals)

    def frobenius_norm(self) -> float:
        s = float(torch.sum(self.vals.double() ** 2).item())
        return math.sqrt(self.pb.comm.allreduce_scalar(s))

    def _spmv(self, beg, end, x, y, acc):
        pb = self.pb
        if pb.platform == "gpu":
            pb.kernels.spmv(self.nrows, beg, end, self.cols, self.vals, x, y, acc)
        else:
            getattr(native.host(), f"bdx_cpu_spmv_{pb.suf}")(
                self.nrows, ptr(beg.numpy()), ptr(end.numpy()), ptr(self.cols.numpy()),
                ptr(self.vals.numpy()), ptr(x.numpy()), ptr(y.numpy()), int(acc))

    def apply(self, x: torch.Tensor, y: torch.Tensor) -> None:
        """y = A x: owned-column pass while the forward exchange is in
        flight, ghost-column pass after it, reverse exchange of ghost rows."""
        pb = self.pb
        work = pb.halo.forward_begin(x)
        self._spmv(self.row_ptr[:-1], self.off, x, y, False)
        pb.halo.forward_end(x, work)
        self._spmv(self.off, self.row_ptr[1:], x, y, True)
        pb.halo.reverse(y)
