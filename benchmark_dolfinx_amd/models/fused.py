"""Fused structured GPU operator (the fast path; csrc/hip/lap_fused.h).

Operator semantics are those of `MatFreeLaplacianGPU` (reference
MatFreeLaplacianGPU, src/laplacian.hpp:87-448) but the whole CG iteration
is restructured around one kernel (see lap_fused.h for the design):

  iteration k:  [halo fwd of r]  fused(p = r + beta p_old, y = A p, p.y partials)
                -> finalize (fold tile-interface partials into y)
                -> [halo rev of y] -> reduce p.y -> [all-reduce]
                -> x += a p, r -= a y, r.r -> [all-reduce]

versus the reference's fill + pack/unpack x2 + 2 stiffness launches + 2
Thrust reductions (host round trips) + 3 axpy launches.
"""

from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

from ..ops import native
from ..ops.kernels import _check, _stream
from ..ops.native import ptr
from ..utils.timing import timed


def fused_supported(pb, version: int = 1) -> bool:
    if pb.platform != "gpu":
        return False
    lib = native.hip()
    if version == 3 and pb.tables.is_identity:
        return False  # fused3 is the phi0 != I core
    if version == 5 and not pb.all_axis_aligned:
        return False  # the Kronecker core needs a diagonal Jacobian per cell
    v = "" if version == 1 else str(version)
    return hasattr(lib, f"bdx_fused{v}_apply_{pb.suf}_p{pb.degree}")


class FusedLaplacianGPU:
    """version=1: lap_fused.h (OTF or stored G); version=2: lap_fused2.h
    (OTF only, precomputed per-thread addressing); version=3: lap_fused3.h
    (fused2 + direct-gradient contraction core, phi0 != I only); version=5:
    lap_fused5.h (nodal Kronecker sum factorisation for axis-aligned box
    cells, P = 3..7, FP64 / FP32)."""

    def __init__(self, pb, geometry: str = "otf", version: int = 1, affine: bool = True,
                 runtime: str = "native", xtri: bool | None = None):
        if geometry not in ("otf", "stored"):
            raise ValueError(f"unknown geometry mode {geometry}")
        if version >= 2 and geometry != "otf":
            raise ValueError("fused2/3 support on-the-fly geometry only")
        if version == 1 and pb.kc is not None:
            raise ValueError("the fused v1 kernel has no per-cell coefficients; use fused2/3 or v1")
        self.version = version
        # CG loop driver for fused2/3: "native" = C++ runtime (solvers/native.py),
        # "python" = the launch sequence below driven from Python
        self.runtime = runtime if version >= 2 else "python"
        self._rt = None
        # fused2: constant-Jacobian kernel instance when every local cell is a
        # parallelepiped (bitwise edge check on the host); else the trilinear one
        self.affine = bool(affine and pb.all_affine)
        if version == 5 and not (self.affine and pb.all_axis_aligned):
            raise ValueError("fused5 needs axis-aligned box cells (diagonal Jacobian)")
        # kernel-instance selector passed as `affine_ok`: fused5 runs on
        # axis-aligned boxes only (2: diagonal Jacobians)
        self.affine_code = int(self.affine)
        if version == 5:
            self.affine_code = 2
        # fused2/3 take 2 on x-trilinear meshes (y/z on the lattice, the
        # reference's --geom_perturb_fact class): the 16-operation per-point
        # geometry instead of the general trilinear one (BDX_F3_XTRI=0: off)
        xtri = affine if xtri is None else xtri
        self.x_trilinear = bool(version in (2, 3) and xtri and not self.affine and pb.all_x_trilinear
                                and os.environ.get("BDX_F3_XTRI", "1") != "0")
        if self.x_trilinear:
            self.affine_code = 2
        if version >= 2:
            geometry = ("otf-affine" if self.affine else
                        "otf-xtrilinear" if self.x_trilinear else "otf-general")
        self.name = "fused" if version == 1 else f"fused{version}"
        self.pb = pb
        self.geometry = geometry
        self.lib = native.hip()
        lat = pb.lat
        t = pb.kernels.t
        self.t = t
        ty, tz = ctypes.c_int(0), ctypes.c_int(0)
        if version == 5:
            _check(getattr(self.lib, f"bdx_fused5_tile_p{pb.degree}_{pb.suf}")(
                self.affine_code, ctypes.byref(ty), ctypes.byref(tz)), "fused5_tile")
        else:
            _check(self.lib.bdx_fused_tile(t.nq, ctypes.byref(ty), ctypes.byref(tz)),
                   "fused_tile")
        self.TY, self.TZ = ty.value, tz.value
        P = lat.degree
        self.nty = max(1, math.ceil(lat.n[1] / self.TY))
        self.ntz = max(1, math.ceil(lat.n[2] / self.TZ))
        self.sy, self.sz = self.TY * P, self.TZ * P
        Lx, Ly, Lz = lat.L
        dev, dt = pb.device, pb.dtype
        self.yb = torch.zeros(max(1, Lx * (self.nty - 1) * Lz), dtype=dt, device=dev)
        self.zb = torch.zeros(max(1, Lx * Ly * (self.ntz - 1)), dtype=dt, device=dev)
        self.cb = torch.zeros(max(1, Lx * (self.nty - 1) * (self.ntz - 1)), dtype=dt, device=dev)
        # x segments per tile (work items = tiles x segments, see
        # fused_set_segments in lap_fused2.h): sized against the chip's
        # resident workgroups so the last round of the launch is not nearly
        # empty.  BDX_SEGMENTS=<n> forces n (1 = whole-x marches).
        self.nseg = 1
        seg_fn = {2: f"bdx_fused2_segments_{pb.suf}_p{pb.degree}",
                  3: f"bdx_fused3_segments_{pb.suf}_p{pb.degree}",
                  5: f"bdx_fused5_segments_{pb.suf}_p{pb.degree}"}.get(version)
        if seg_fn and hasattr(self.lib, seg_fn):
            forced = os.environ.get("BDX_SEGMENTS", "")
            args = (self.nty * self.ntz, lat.n[0])
            if version == 5:
                args = (self.affine_code,) + args
            elif version in (2, 3):
                args = (self.affine_code, t.nq) + args
            self.nseg = int(forced) if forced else int(getattr(self.lib, seg_fn)(*args))
            self.nseg = max(1, min(self.nseg, max(1, lat.n[0])))
            seglen = -(-lat.n[0] // self.nseg)
            self.nseg = -(-lat.n[0] // seglen)  # no empty segments (as the kernel)
        self.nblocks = self.nty * self.ntz * self.nseg
        self.partials = torch.zeros(self.nblocks, dtype=torch.float64, device=dev)
        self.G = None
        if geometry == "stored":
            with timed("~setup geometry"):
                self.G = torch.empty(lat.ncells_local * 6 * t.nq ** 3, dtype=dt, device=dev)
                pb.kernels.geometry(pb.xv, self.G)
        # packed 1D tables (uniform rows are read through scalar loads)
        if version == 5:
            # 1D mass / stiffness / mixed matrices of the quadrature rule, in T
            self._Dd = np.ascontiguousarray(pb.tables.Dd, dtype=np.float64)
            ftab5 = getattr(self.lib, f"bdx_fused5_tables_{pb.suf}_p{pb.degree}")
            wts = np.ascontiguousarray(t.wts, dtype=np.float64)
            ntab = ftab5(t.nd, t.nq, ptr(t.phi0), ptr(self._Dd), ptr(wts), None)
            if ntab <= 0:
                raise RuntimeError(f"no fused5 tables for nd={t.nd} nq={t.nq}")
            host = np.zeros(ntab, dtype=np.float64 if pb.dtype == torch.float64 else np.float32)
            ftab5(t.nd, t.nq, ptr(t.phi0), ptr(self._Dd), ptr(wts), ptr(host))
        else:
            if version == 3:
                self._Dd = np.ascontiguousarray(pb.tables.Dd, dtype=np.float64)
                ftab = getattr(self.lib, f"bdx_fused3_tables_{pb.suf}")
                second = self._Dd
            else:
                ftab = getattr(self.lib, f"bdx_fused_tables_{pb.suf}")
                second = t.dphi1
            ntab = ftab(t.nd, t.nq, ptr(t.phi0), ptr(second), None)
            if ntab <= 0:
                raise RuntimeError(f"no fused tables for nd={t.nd} nq={t.nq}")
            host = np.zeros(ntab, dtype=np.float64 if pb.dtype == torch.float64 else np.float32)
            ftab(t.nd, t.nq, ptr(t.phi0), ptr(second), ptr(host))
        if version == 5:
            # fused5 reads its tables through a pointer: a device buffer owned
            # by this operator (a captured graph keeps reading its own tables)
            self.tabs_host = host
            self.tabs = torch.from_numpy(host).to(dev)
        else:
            self.tabs = host  # host memory: copied into the kernel arguments
        if version >= 2:
            self._apply2 = getattr(self.lib, f"bdx_fused{version}_apply_{pb.suf}_p{P}")
        else:
            self._apply = getattr(self.lib, f"bdx_fused_apply_{pb.suf}_p{P}")
        self._final = getattr(self.lib, f"bdx_fused_finalize_{pb.suf}")
        self.geom_code = 1 if geometry == "otf" else 0
        self.p_old = None
        self.p_new = None

    def close(self) -> None:
        """Release the native runtime (RCCL communicator, graphs, stream)
        before the process group / HIP runtime shut down."""
        if self._rt is not None:
            self._rt.close()
            self._rt = None

    # ------------------------------------------------------------ launches
    def _finalize(self, y, ghost_only: bool = False):
        _check(self._final(ptr(self.pb.latd), ptr(y), ptr(self.yb), ptr(self.zb), ptr(self.cb),
                           self.nty, self.ntz, self.sy, self.sz, int(ghost_only), _stream()),
               "fused_finalize")

    def _launch(self, mode, u, pold, pnew, y, scal=None, beta_num=-1, beta_den=-1, x=None,
                xa_num=-1, xa_den=-1, finalize=True):
        pb, t = self.pb, self.t
        if self.version >= 2:
            _check(self._apply2(mode | (self.nseg << 8), self.affine_code, ptr(pb.latd), t.nq,
                                ptr(t.wts),
                                ptr(t.qpts), ptr(u), ptr(pold), ptr(pnew), ptr(x), ptr(y),
                                ptr(self.yb), ptr(self.zb), ptr(self.cb), ptr(pb.xv),
                                ptr(pb.kc), ptr(self.tabs), pb.kappa, ptr(scal), ptr(self.partials),
                                beta_num, beta_den, xa_num, xa_den, self.nty, self.ntz, None,
                                _stream()), "fused2_apply")
        else:
            _check(self._apply(self.geom_code, mode, ptr(pb.latd), t.nq, ptr(t.phi0),
                               ptr(t.dphi1), ptr(t.wts), ptr(t.qpts), ptr(u), ptr(pold),
                               ptr(pnew), ptr(y), ptr(self.yb), ptr(self.zb), ptr(self.cb),
                               ptr(self.G), ptr(pb.xv), ptr(self.tabs), pb.kappa, ptr(scal),
                               ptr(self.partials), beta_num, beta_den, self.nty, self.ntz,
                               _stream()), "fused_apply")
        if finalize:
            self._finalize(y)

    def apply(self, u: torch.Tensor, y: torch.Tensor) -> None:
        """y = A u (action mode)."""
        halo = self.pb.halo
        halo.forward(u)
        self._launch(0, u, None, None, y)
        halo.reverse(y)

    # ------------------------------------------------------------- CG
    def cg_start(self, cg, x, b):
        k, r, y = cg.k, cg.r, cg.y
        self.apply(x, y)
        k.axpy(r, -1.0, y, b)
        k.dot(r, r, cg.partials, cg.scal, cg.RR0)
        cg._allreduce(cg.RR0)
        if self.p_old is None:
            self.p_old = self.pb.new_vector()
            self.p_new = self.pb.new_vector()
        else:
            self.p_old.zero_()
        self.x_lag = False
        self._own = np.array(self.pb.lat.owned_hi, dtype=np.int64)
        if self.runtime == "native":
            if self._rt is None or self._rt.cg is not cg:
                from ..solvers.native import NativeCGRuntime, NativeRuntimeUnavailable
                if self._rt is not None:
                    self._rt.close()
                try:
                    self._rt = NativeCGRuntime(self, cg)
                except NativeRuntimeUnavailable as e:
                    # raised on every rank alike (construction is collective),
                    # so all ranks take the Python driver of the same kernels
                    import sys
                    print(f"[bdx] native CG runtime unavailable ({e}); using the Python "
                          f"driver of the same kernels", file=sys.stderr)
                    self.runtime, self._rt = "python", None
            if self._rt is not None:
                self._rt.bind_x(x)  # DeviceCG.start may pass another iterate
                self._rt.reset()

    def cg_iterate(self, cg, n, flush=True):
        if self.version >= 2 and self._rt is not None:
            return self._rt.iterate(n)
        if self.version >= 2:
            return self._cg_iterate2(cg, n, flush)
        k, r, y, x, scal = cg.k, cg.r, cg.y, cg.x, cg.scal
        halo = self.pb.halo
        for _ in range(n):
            cur = cg.RR0 if cg.it % 2 == 0 else cg.RR1
            nxt = cg.RR1 if cg.it % 2 == 0 else cg.RR0
            halo.forward(r)
            bnum, bden = (cur, nxt) if cg.it > 0 else (-1, -1)
            self._launch(1, r, self.p_old, self.p_new, y, scal, bnum, bden)
            halo.reverse(y)
            _check(self.lib.bdx_reduce_partials(ptr(self.partials), self.nblocks, ptr(scal),
                                                cg.PAP, _stream()), "reduce_partials")
            cg._allreduce(cg.PAP)
            k.cg_update(x, r, self.p_new, y, scal, cur, cg.PAP, nxt, cg.partials)
            cg._allreduce(nxt)
            self.p_old, self.p_new = self.p_new, self.p_old
            cg.it += 1

    def _cg_iterate2(self, cg, n, flush=True):
        """fused2 CG iteration: x += alpha_prev p_old rides in the fused
        kernel's staging (lagged one iteration, flushed at the end); the tile
        interface partials are folded inside the r update (no finalize pass
        over y; with several ranks only the ghost planes are finalized, before
        the reverse halo packs them)."""
        r, y, x, scal = cg.r, cg.y, cg.x, cg.scal
        pb = self.pb
        halo = pb.halo
        multi = halo.active
        upd = getattr(self.lib, f"bdx_cg_update_iface_{pb.suf}")
        for _ in range(n):
            cur = cg.RR0 if cg.it % 2 == 0 else cg.RR1
            nxt = cg.RR1 if cg.it % 2 == 0 else cg.RR0
            halo.forward(r)
            bnum, bden = (cur, nxt) if cg.it > 0 else (-1, -1)
            xnum, xden = (nxt, cg.PAP) if self.x_lag else (-1, -1)
            self._launch(1, r, self.p_old, self.p_new, y, scal, bnum, bden, x, xnum, xden,
                         finalize=False)
            if multi:
                self._finalize(y, ghost_only=True)
                halo.reverse(y)
            _check(self.lib.bdx_reduce_partials(ptr(self.partials), self.nblocks, ptr(scal),
                                                cg.PAP, _stream()), "reduce_partials")
            cg._allreduce(cg.PAP)
            _check(upd(ptr(pb.latd), ptr(self._own), ptr(r), ptr(y), ptr(self.yb),
                       ptr(self.zb), ptr(self.cb), self.nty, self.ntz, self.sy, self.sz,
                       ptr(scal), cur, cg.PAP, nxt, ptr(cg.partials), _stream()),
                   "cg_update_iface")
            cg._allreduce(nxt)
            self.p_old, self.p_new = self.p_new, self.p_old
            self.x_lag = True
            cg.it += 1
        if flush:
            self.flush_x(cg)

    def flush_x(self, cg):
        """Apply the pending x += alpha_last p_last of the lagged update."""
        if not self.x_lag:
            return
        last = cg.RR0 if (cg.it - 1) % 2 == 0 else cg.RR1
        _check(getattr(self.lib, f"bdx_xflush_{self.pb.suf}")(
            ptr(self.pb.latd), ptr(self._own), ptr(cg.x), ptr(self.p_old), ptr(cg.scal), last,
            cg.PAP, _stream()), "xflush")
        self.x_lag = False
