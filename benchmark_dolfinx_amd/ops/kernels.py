"""Python front-end of the HIP kernels: torch tensors in, kernels on the
current HIP stream, errors raised loudly (no silent fallback)."""

from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import native
from .native import ptr


def _suf(dtype) -> str:
    if dtype == torch.float64:
        return "f64"
    if dtype == torch.float32:
        return "f32"
    raise TypeError(f"unsupported dtype {dtype}")


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


class HipError(RuntimeError):
    pass


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise HipError(f"{what} failed with hipError {rc}")


class TableSet:
    """float64 copies of the 1D tables kept alive for ctypes calls."""

    def __init__(self, tables):
        self.nq = tables.nq
        self.nd = tables.nd
        self.identity = int(tables.is_identity)
        self.phi0 = np.ascontiguousarray(tables.phi0, dtype=np.float64)
        self.dphi1 = np.ascontiguousarray(tables.dphi1, dtype=np.float64)
        self.wts = np.ascontiguousarray(tables.qwts, dtype=np.float64)
        self.qpts = np.ascontiguousarray(tables.qpts, dtype=np.float64)


class HipKernels:
    """Bound kernel launchers for one problem (lattice + tables + dtype)."""

    def __init__(self, lat, tables, dtype):
        self.lib = native.hip()
        self.lat = lat
        self.latd = lat.as_int64()
        self.t = TableSet(tables)
        self.dtype = dtype
        self.suf = _suf(dtype)
        self.npart = self.lib.bdx_hip_partials_size()
        self.o = lat.owned_hi

    def _f(self, name):
        return getattr(self.lib, f"{name}_{self.suf}")

    # --------------------------------------------------------------- operator
    def v1_apply(self, mode: int, G, xv, kappa: float, u, y, lo, hi, kc=None):
        lo = np.asarray(lo, dtype=np.int64)
        hi = np.asarray(hi, dtype=np.int64)
        t = self.t
        _check(self._f("bdx_v1_apply")(mode, ptr(self.latd), t.nq, ptr(t.phi0),
                                       ptr(t.dphi1), ptr(t.wts), ptr(t.qpts), t.identity,
                                       ptr(G), ptr(xv), kappa, ptr(kc), ptr(u), ptr(y), ptr(lo),
                                       ptr(hi), _stream()), "v1_apply")

    def dofmap_tables(self, device):
        """Device copy of the 1D tables the dofmap kernels read:
        [phi0 (nq x nd) | dphi1 (nq x nq) | qpts | wts | Dd = dphi1 phi0 (nq x nd) |
        phi0^T | Dd^T] in the vector dtype (Dd and the transposes: the MFMA kernel,
        lap_dofmfma.h)."""
        t = self.t
        dd = np.asarray(t.dphi1, dtype=np.float64) @ np.asarray(t.phi0, dtype=np.float64)
        h = np.concatenate([t.phi0.ravel(), t.dphi1.ravel(), t.qpts.ravel(), t.wts.ravel(),
                            dd.ravel(), np.ascontiguousarray(t.phi0.T).ravel(),
                            np.ascontiguousarray(dd.T).ravel()])
        return torch.from_numpy(h).to(device, self.dtype)

    def dofmap_apply(self, geom: int, tab, cells, ncl: int, cdofs, cverts, coords, flags, G,
                     kappa: float, kc, u, y, mode: int = 0, pold=None, pnew=None, x=None,
                     scal=None, beta=(-1, -1), xa=(-1, -1), partials=None) -> int:
        """mode 0: y += A u; 1: the CG operator (u = r; see lap_dofmap.h).
        Returns the number of p.Ap partials written (CG)."""
        t, P = self.t, self.lat.degree
        nb = ctypes.c_int(0)
        nvec = int(u.numel())
        if nvec * u.element_size() >= 2 ** 32 - 16:
            raise ValueError("dofmap operator: vectors beyond 4 GiB exceed the 32-bit buffer range")
        _check(self._f("bdx_dofmap_apply")(P, t.nq, geom, mode, ptr(tab), ptr(cells), ncl, nvec,
                                           ptr(cdofs), ptr(cverts), ptr(coords), ptr(flags),
                                           ptr(G), kappa, ptr(kc), ptr(u), ptr(pold), ptr(pnew),
                                           ptr(x), ptr(y), ptr(scal), beta[0], beta[1], xa[0],
                                           xa[1], ptr(partials), ctypes.byref(nb), _stream()),
               "dofmap_apply")
        return nb.value

    def dofmap_cg_update(self, flags, r, y, scal, rn_slot: int, pap_slot: int, partials) -> int:
        nb = ctypes.c_int(0)
        _check(self._f("bdx_dofmap_cg_update")(r.numel(), ptr(flags), ptr(r), ptr(y), ptr(scal),
                                               rn_slot, pap_slot, ptr(partials), ctypes.byref(nb),
                                               _stream()), "dofmap_cg_update")
        return nb.value

    def dofmap_xflush(self, x, p, scal, num: int, den: int):
        _check(self._f("bdx_dofmap_xflush")(x.numel(), ptr(x), ptr(p), ptr(scal), num, den,
                                            _stream()), "dofmap_xflush")

    def dofmap_mark_writers(self, cells_a, cells_b, cdofs, nd3: int, ndofs: int):
        first = torch.empty(max(1, ndofs), dtype=torch.int32, device=cdofs.device)
        _check(self.lib.bdx_dofmap_mark_writers(ptr(cells_a), int(cells_a.numel()), ptr(cells_b),
                                                int(cells_b.numel()), ptr(cdofs), nd3, ptr(first),
                                                ndofs, _stream()), "dofmap_mark_writers")

    def reduce_partials(self, partials, n: int, out, slot: int):
        _check(self.lib.bdx_reduce_partials(ptr(partials), n, ptr(out), slot, _stream()),
               "reduce_partials")

    def dofmap_geometry(self, ncells: int, cverts, coords, G):
        t, P = self.t, self.lat.degree
        _check(self._f("bdx_dofmap_geometry")(P, t.nq, ptr(t.phi0), ptr(t.dphi1), ptr(t.wts),
                                              ptr(t.qpts), ncells, ptr(cverts), ptr(coords),
                                              ptr(G), _stream()), "dofmap_geometry")

    def geometry(self, xv, G):
        t = self.t
        _check(self._f("bdx_geometry")(ptr(self.latd), t.nq, ptr(t.phi0), ptr(t.dphi1),
                                       ptr(t.wts), ptr(t.qpts), ptr(xv), ptr(G), _stream()),
               "geometry")

    # ------------------------------------------------------------------ BLAS
    def dot(self, a, b, partials, out, slot: int):
        L = self.lat
        _check(self._f("bdx_dot")(L.L[1], L.ld, self.o[0], self.o[1], self.o[2], ptr(a),
                                  ptr(b), ptr(partials), ptr(out), slot, _stream()), "dot")

    def cg_update(self, x, r, p, y, scal, rn_slot, pap_slot, out_slot, partials):
        L = self.lat
        _check(self._f("bdx_cg_update")(L.L[1], L.ld, self.o[0], self.o[1], self.o[2],
                                        ptr(x), ptr(r), ptr(p), ptr(y), ptr(scal), rn_slot,
                                        pap_slot, out_slot, ptr(partials), _stream()),
               "cg_update")

    def p_update(self, p, r, scal, num, den):
        L = self.lat
        _check(self._f("bdx_p_update")(L.L[1], L.ld, self.o[0], self.o[1], self.o[2],
                                       ptr(p), ptr(r), ptr(scal), num, den, _stream()),
               "p_update")

    def axpy(self, out, alpha: float, x, y):
        L = self.lat
        _check(self._f("bdx_axpy")(L.L[1], L.ld, self.o[0], self.o[1], self.o[2], ptr(out),
                                   float(alpha), ptr(x), ptr(y), _stream()), "axpy")

    def box_copy(self, mode: int, vec, lat, side, buf):
        _check(self._f("bdx_box_copy")(mode, ptr(vec), lat.L[1], lat.ld, ptr(side.table),
                                       len(side.boxes), side.total, ptr(buf), _stream()),
               "box_copy")

    def spmv(self, nrows, beg, end, cols, vals, x, y, acc=False):
        """y[r] (+)= sum of vals[p] x[cols[p]] over p in [beg[r], end[r])."""
        _check(self._f("bdx_spmv")(nrows, ptr(beg), ptr(end), ptr(cols), ptr(vals), ptr(x),
                                   ptr(y), int(acc), _stream()), "spmv")


def device_info(dev: int = 0) -> str:
    import ctypes
    lib = native.hip()
    buf = ctypes.create_string_buffer(1024)
    rc = lib.bdx_device_info(dev, buf, 1024)
    if rc != 0:
        return f"(device info unavailable: hipError {rc})\n"
    return buf.value.decode()


def device_name(dev: int = 0) -> str:
    """hipDeviceProp name + gcnArchName (torch's get_device_name() returns a
    generic marketing string on this stack)."""
    info = device_info(dev)
    fields = {}
    for line in info.splitlines():
        key, sep, val = line.partition(":")
        if sep:
            fields[key.strip()] = val.strip()
    name = fields.get("Device", "unknown")
    arch = fields.get("gcnArch", "")
    return f"{name} ({arch})" if arch else name
