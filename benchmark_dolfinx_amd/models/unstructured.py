"""Unstructured (dofmap) data model and its GPU operator.

The reference stores a mesh the DOLFINx way: an explicit cell -> dof map, a
cell -> geometry-node map with node coordinates, per-dof boundary markers and
(for the GPU operator) per-quadrature-point geometry G, and it applies the
operator through that indirection (src/laplacian.hpp:105-114,
src/laplacian_gpu.hpp:153-170, built from the mesh in src/mesh.cpp:87-102;
interior / boundary cell lists for the overlapped schedule,
src/laplacian.hpp:215-272 and :281-349).

`UnstructuredMesh` is that representation.  `from_problem` builds it for the
benchmark's box (the lattice is only used to *construct* the arrays); nothing
downstream assumes a lattice, so any hexahedral mesh, cell order or dof
numbering can be fed in (`renumbered` applies arbitrary permutations and the
tests check the operator is equivariant under them).  `DofmapLaplacianGPU`
runs the `lap_dofmap` HIP kernel (csrc/hip/lap_dofmap.h): a wave-local
line-per-lane sum factorisation behind the dofmap gather and an atomic
scatter-add, with the same interior-then-boundary overlap of the forward halo
exchange as the reference, and a fused CG iteration.  Vectors keep the problem's storage layout, so the halo machinery
and the CG solvers are shared with the structured operators.
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
import torch

from ..utils.timing import timed


@dataclass
class UnstructuredMesh:
    cell_dofs: np.ndarray        # int32 [ncells, nd^3], tensor-product order (i, j, k)
    cell_verts: np.ndarray       # int32 [ncells, 8], v = 4a + 2b + c
    coords: np.ndarray           # [nverts, 3] geometry nodes
    dof_flags: np.ndarray        # uint8 [ndofs]: bit 0 Dirichlet, bit 1 owned
    interior_cells: np.ndarray   # int32: cells touching no ghost dof
    boundary_cells: np.ndarray   # int32: the rest (computed after the halo arrives)
    kc: np.ndarray | None        # per-cell coefficient or None (constant kappa)
    degree: int

    @property
    def ncells(self) -> int:
        return int(self.cell_dofs.shape[0])

    @property
    def ndofs(self) -> int:
        return int(self.dof_flags.shape[0])

    @classmethod
    def from_problem(cls, pb) -> "UnstructuredMesh":
        """The dofmap arrays of the problem's local box (cell id = the
        lexicographic cell index of the lattice, dof id = the storage index)."""
        lat = pb.lat
        P, nd = lat.degree, lat.degree + 1
        n0, n1, n2 = lat.n
        L1, ld = lat.L[1], lat.ld
        cx, cy, cz = np.meshgrid(np.arange(n0, dtype=np.int64), np.arange(n1, dtype=np.int64),
                                 np.arange(n2, dtype=np.int64), indexing="ij")
        cx, cy, cz = cx.ravel(), cy.ravel(), cz.ravel()
        nc = cx.size
        cdofs = np.empty((nc, nd ** 3), dtype=np.int32)
        for i in range(nd):
            for j in range(nd):
                for k in range(nd):
                    cdofs[:, (i * nd + j) * nd + k] = (((cx * P + i) * L1 + cy * P + j) * ld
                                                       + cz * P + k)
        cverts = np.empty((nc, 8), dtype=np.int32)
        for v in range(8):
            a, b, c = v >> 2, (v >> 1) & 1, v & 1
            cverts[:, v] = ((cx + a) * (n1 + 1) + cy + b) * (n2 + 1) + cz + c
        flags = np.zeros(lat.shape, dtype=np.uint8)
        L = lat.L
        flags[:L[0], :L[1], :L[2]] = (lat.bc_mask().astype(np.uint8)
                                      | (lat.owned_mask().astype(np.uint8) << 1))
        hi = [m - g for m, g in zip(lat.n, lat.gh)]
        inner = (cx < hi[0]) & (cy < hi[1]) & (cz < hi[2])
        ids = np.arange(nc, dtype=np.int32)
        return cls(cdofs, cverts, np.ascontiguousarray(pb.xv_host.reshape(-1, 3)),
                   flags.ravel(), ids[inner], ids[~inner],
                   None if pb.kc is None else np.ascontiguousarray(pb.kc_host.reshape(-1)), P)

    def renumbered(self, dof_perm: np.ndarray | None = None,
                   cell_perm: np.ndarray | None = None,
                   vert_perm: np.ndarray | None = None) -> "UnstructuredMesh":
        """The same mesh with dof i renamed dof_perm[i], cell c stored at row
        position where cell_perm[pos] = c, vertex v renamed vert_perm[v]."""
        cd, cv, co, fl, kc = self.cell_dofs, self.cell_verts, self.coords, self.dof_flags, self.kc
        inner, outer = self.interior_cells, self.boundary_cells
        if dof_perm is not None:
            cd = dof_perm[cd].astype(np.int32)
            fl = np.empty_like(fl)
            fl[dof_perm] = self.dof_flags
        if vert_perm is not None:
            cv = vert_perm[cv].astype(np.int32)
            co = np.empty_like(co)
            co[vert_perm] = self.coords
        if cell_perm is not None:
            pos = np.empty_like(cell_perm)
            pos[cell_perm] = np.arange(cell_perm.size)
            cd, cv = cd[cell_perm], cv[cell_perm]
            kc = None if kc is None else kc[cell_perm]
            inner, outer = np.sort(pos[inner]).astype(np.int32), np.sort(pos[outer]).astype(np.int32)
        return UnstructuredMesh(np.ascontiguousarray(cd), np.ascontiguousarray(cv),
                                np.ascontiguousarray(co), fl, inner, outer,
                                None if kc is None else np.ascontiguousarray(kc), self.degree)


class DofmapLaplacianGPU:
    """Matrix-free stiffness operator on the unstructured data model.

    geometry="otf": G per quadrature point from the cell's 8 geometry nodes;
    "stored": G precomputed once per (cell, point) in the reference layout
    [cell][6][nq^3] (src/geometry_gpu.hpp:26-132).

    `apply` is the reference's operator action.  Under DeviceCG the operator
    runs its own fused CG iteration (`cg_start` / `cg_iterate`,
    csrc/hip/lap_dofmap.h): p = r + beta p_old, the lagged x update and the
    p.Ap element dots ride in the gather / scatter of the operator kernel, and
    one update pass does r -= alpha y, r.r and y = 0 -- the reference's five
    BLAS-1 calls per iteration (src/cg.hpp:121-167) become one.  The
    iteration loop runs in the native C++ runtime (runtime.hip DofCGRuntime:
    interior cells on the compute stream, forward exchange -> boundary cells
    -> reverse send on the comm stream, device all-reduces, watchdog);
    `runtime="python"` (or BDX_DOFMAP_RUNTIME=python) drives the same kernels
    from Python with torch collectives.
    """

    name = "dofmap"
    RR0, RR1, PAP = 0, 1, 2  # DeviceCG's scalar slots

    def __init__(self, problem, geometry: str = "otf", mesh: UnstructuredMesh | None = None,
                 runtime: str | None = None):
        if problem.platform != "gpu":
            raise ValueError("DofmapLaplacianGPU needs the GPU platform")
        if geometry not in ("otf", "stored"):
            raise ValueError(f"unknown geometry mode {geometry}")
        self.pb = problem
        self.k = problem.kernels
        self.geometry = f"dofmap-{geometry}"
        with timed("~setup dofmap"):
            self.mesh = mesh or UnstructuredMesh.from_problem(problem)
            dev, dt = problem.device, problem.dtype
            m = self.mesh
            self.cdofs = torch.from_numpy(m.cell_dofs).to(dev)
            self.cverts = torch.from_numpy(m.cell_verts).to(dev)
            self.coords = torch.from_numpy(m.coords).to(dev, dt)
            self.flags = torch.from_numpy(m.dof_flags).to(dev)
            self.tab = self.k.dofmap_tables(dev)
            if os.environ.get("BDX_TEST_CORRUPT_DOFMAP"):
                # test hook (tests/test_gpu_bench_consistency.py): a 0.1 % error
                # in one interpolation entry, which bench.py's cross-family
                # consistency gate must catch
                self.tab[0] *= 1.001
            self.inner = torch.from_numpy(m.interior_cells).to(dev)
            self.outer = torch.from_numpy(m.boundary_cells).to(dev)
            self.kc = None if m.kc is None else torch.from_numpy(m.kc).to(dev, dt)
            # writer designation (sign bit of cell_dofs): the first occurrence
            # of each dof in launch order (interior cells, then boundary cells)
            self.k.dofmap_mark_writers(self.inner, self.outer, self.cdofs,
                                       int(m.cell_dofs.shape[1]), m.ndofs)
            self.G = None
            self.geom = 1
            if geometry == "stored":
                nq3 = problem.tables.nq ** 3
                self.G = torch.empty(m.ncells * 6 * nq3, dtype=dt, device=dev)
                self.k.dofmap_geometry(m.ncells, self.cverts, self.coords, self.G)
                self.geom = 0
        # the FP64 operator kernel the launches take (lap_dofmap.h: the VALU
        # line-per-lane kernel by default, lap_dofmfma.h's MFMA one under
        # BDX_DOFMAP_MFMA=1 / bdx_dofmap_set_mfma); FP32 is always VALU
        nd, nq = problem.tables.nd, problem.tables.nq
        self.core = ("mfma" if dt == torch.float64 and self.k.lib.bdx_dofmap_uses_mfma(nd, nq)
                     else "valu")
        self._cg = None
        self._rt = None
        # native (default) at every rank count.  Its multi-rank split schedule
        # is verified with thread ranks on one GPU (tests/test_gpu_dofmap.py)
        # and shares the RCCL transport of the fused runtime; a run of it on
        # separate GPUs has not been recorded yet (docs/PARITY.md).
        # BDX_DOFMAP_RUNTIME=python selects the Python driver.
        self.runtime = runtime or os.environ.get("BDX_DOFMAP_RUNTIME", "native")

    def close(self) -> None:
        """Release the native runtime (RCCL communicator, streams)."""
        if self._rt is not None:
            self._rt.close()
            self._rt = None

    def _run(self, cells, u, y, **kw) -> int:
        n = int(cells.numel())
        if not n:
            return 0
        return self.k.dofmap_apply(self.geom, self.tab, cells, n, self.cdofs, self.cverts, self.coords,
                                   self.flags, self.G, self.pb.kappa, self.kc, u, y, **kw)

    def apply(self, u: torch.Tensor, y: torch.Tensor) -> None:
        pb = self.pb
        y.zero_()
        work = pb.halo.forward_begin(u)
        self._run(self.inner, u, y)      # overlaps the forward exchange
        pb.halo.forward_end(u, work)
        self._run(self.outer, u, y)
        pb.halo.reverse(y)

    # ------------------------------------------------------------ fused CG
    def cg_start(self, cg, x, b):
        """r0 = b - A x0, rho0 = r0.r0 (owned), p_old = 0, y = 0."""
        pb, k = self.pb, self.k
        self.apply(x, cg.y)
        k.axpy(cg.r, -1.0, cg.y, b)
        k.dot(cg.r, cg.r, cg.partials, cg.scal, self.RR0)
        cg._allreduce(self.RR0)
        n = pb.lat.nstore
        if getattr(self, "p_a", None) is None:
            # allocated once: the native runtime keeps pointers to them
            self.p_a = torch.zeros(n, dtype=pb.dtype, device=pb.device)
            self.p_b = torch.zeros(n, dtype=pb.dtype, device=pb.device)
            self.part = torch.zeros(int(cg.partials.numel()), dtype=torch.float64,
                                    device=pb.device)
        else:
            self.p_a.zero_()  # p_old of the first iteration (beta = 0 still reads it)
        cg.y.zero_()
        self.x_lag = False
        self._cg = cg
        if self.runtime == "native":
            if self._rt is None or self._rt.cg is not cg:
                from ..solvers.native import NativeCGRuntime, NativeRuntimeUnavailable
                if self._rt is not None:
                    self._rt.close()
                try:
                    self._rt = NativeCGRuntime(self, cg)
                except NativeRuntimeUnavailable as e:
                    import sys
                    print(f"[bdx] native CG runtime unavailable ({e}); using the Python "
                          f"driver of the dofmap kernels", file=sys.stderr)
                    self.runtime, self._rt = "python", None
            if self._rt is not None:
                self._rt.bind_x(x)
                self._rt.reset()

    def cg_iterate(self, cg, n: int, flush: bool = True) -> None:
        """n fused CG iterations; `flush=False` leaves the last lagged x
        update pending (a later call or `flush` applies it).  The native
        runtime ignores `flush` (as the fused operators' does): its
        iterate() always folds the pending x term at the end of the call,
        so x is current after every call."""
        if self._rt is not None:
            return self._rt.iterate(n)
        pb, k = self.pb, self.k
        r, y, x, scal = cg.r.view(-1), cg.y.view(-1), cg.x.view(-1), cg.scal
        for _ in range(n):
            it = cg.it
            cur, nxt = (self.RR0, self.RR1) if it % 2 == 0 else (self.RR1, self.RR0)
            pold, pnew = (self.p_a, self.p_b) if it % 2 == 0 else (self.p_b, self.p_a)
            kw = dict(mode=1, pold=pold, pnew=pnew, x=x, scal=scal,
                      beta=(-1, -1) if it == 0 else (cur, nxt),
                      xa=(nxt, self.PAP) if self.x_lag else (-1, -1))
            work = pb.halo.forward_begin(cg.r)
            n1 = self._run(self.inner, r, y, partials=self.part, **kw)
            pb.halo.forward_end(cg.r, work)
            n2 = self._run(self.outer, r, y, partials=self.part[n1:], **kw)
            pb.halo.reverse(cg.y)
            k.reduce_partials(self.part, n1 + n2, scal, self.PAP)
            cg._allreduce(self.PAP)
            nu = k.dofmap_cg_update(self.flags, r, y, scal, cur, self.PAP, self.part)
            k.reduce_partials(self.part, nu, scal, nxt)
            cg._allreduce(nxt)
            self.x_lag = True
            cg.it += 1
        if flush:
            self.flush(cg)

    def flush(self, cg) -> None:
        """Apply the lagged x += alpha p of the last iteration."""
        if not self.x_lag:
            return
        last = self.RR0 if (cg.it - 1) % 2 == 0 else self.RR1
        plast = self.p_b if (cg.it - 1) % 2 == 0 else self.p_a
        self.k.dofmap_xflush(cg.x.view(-1), plast, cg.scal, last, self.PAP)
        self.x_lag = False


class DofmapLaplacianCPU:
    """The reference data model on the CPU platform: the C++/OpenMP operator
    gathers through the explicit cell -> dof map with G stored per cell in the
    reference layout [cell][6][nq^3] (the reference's MatFreeLaplacianCPU with
    geometry_computation_cpu, src/laplacian.hpp:450-771,
    src/geometry_cpu.hpp:25-112; 64-bit offsets, quirk Q6), scatters with
    atomic adds and runs the same interior / boundary split around the
    forward halo exchange as the GPU operator.  geometry="otf": per-point
    geometry from the cell vertices instead of stored G."""

    name = "dofmap"

    def __init__(self, problem, geometry: str = "stored", mesh: UnstructuredMesh | None = None):
        from ..ops import native
        if problem.platform != "cpu":
            raise ValueError("DofmapLaplacianCPU runs on the CPU platform")
        if geometry not in ("otf", "stored"):
            raise ValueError(f"unknown geometry mode {geometry}")
        self.pb = problem
        self.geometry = f"dofmap-{geometry}"
        self.lib = native.host()
        suf = problem.suf
        self._fn = getattr(self.lib, f"bdx_cpu_dofmap_{suf}")
        npdt = np.float64 if suf == "f64" else np.float32
        with timed("~setup dofmap"):
            self.mesh = m = mesh or UnstructuredMesh.from_problem(problem)
            self.cdofs = np.ascontiguousarray(m.cell_dofs, dtype=np.int32)
            self.cverts = np.ascontiguousarray(m.cell_verts, dtype=np.int32)
            self.coords = np.ascontiguousarray(m.coords, dtype=npdt)
            self.flags = np.ascontiguousarray(m.dof_flags, dtype=np.uint8)
            self.inner = np.ascontiguousarray(m.interior_cells, dtype=np.int32)
            self.outer = np.ascontiguousarray(m.boundary_cells, dtype=np.int32)
            self.kc = None if m.kc is None else np.ascontiguousarray(m.kc, dtype=npdt)
            t = problem.host_tables
            self.t = t
            self.G = None
            if geometry == "stored":
                nq = problem.tables.nq
                self.G = np.empty(m.ncells * 6 * nq ** 3, dtype=npdt)
                getattr(self.lib, f"bdx_cpu_dofmap_geometry_{suf}")(
                    problem.lat.degree, nq, native.ptr(t["wts"]), native.ptr(t["qpts"]),
                    m.ncells, native.ptr(self.cverts), native.ptr(self.coords),
                    native.ptr(self.G))

    def _run(self, cells, u, y):
        from ..ops.native import ptr
        if cells.size == 0:
            return
        t, pb = self.t, self.pb
        self._fn(pb.lat.degree, pb.tables.nq, ptr(t["phi0"]), ptr(t["dphi1"]), ptr(t["wts"]),
                 ptr(t["qpts"]), int(pb.tables.is_identity), ptr(cells), int(cells.size),
                 ptr(self.cdofs), ptr(self.cverts), ptr(self.coords), ptr(self.G), ptr(self.flags),
                 pb.kappa, ptr(self.kc), ptr(u), ptr(y))

    def apply(self, u: torch.Tensor, y: torch.Tensor) -> None:
        pb = self.pb
        y.zero_()
        work = pb.halo.forward_begin(u)
        self._run(self.inner, u, y)      # overlaps the forward exchange
        pb.halo.forward_end(u, work)
        self._run(self.outer, u, y)
        pb.halo.reverse(y)
