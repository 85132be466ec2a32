"""Python handle of the native C++ CG runtime (csrc/hip/runtime.hip).

After the CG prologue (r0 = b - A x0, rho0 = r0.r0; FusedLaplacianGPU.cg_start)
the whole iteration loop -- halo exchange, fused operator, reductions,
all-reduces, r/x updates -- runs in C++ on the current HIP stream, with the
steady-state iterations replayed from hipGraphs.  Transport:

* ``rccl``   one process per GPU (torchrun); the runtime opens its own RCCL
  communicator, bootstrapped by exchanging an ncclUniqueId over the existing
  torch.distributed group, and exchanges halos with grouped ncclSend/ncclRecv
  to the neighbours only;
* ``thread`` ranks are threads of one process on one GPU (ThreadComm tests);
* single rank: no communication.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from ..ops import native
from ..ops.kernels import _check, _stream
from ..ops.native import ptr


class NativeCGRuntime:
    def __init__(self, op, cg, use_graph: bool | None = None):
        pb = op.pb
        self.op, self.cg, self.pb = op, cg, pb
        self.lib = native.hip()
        comm = pb.comm
        halo = pb.halo
        if use_graph is None:
            # BDX_GRAPH=0 off, 1 (default) single-rank only, 2 also with RCCL
            # (multi-rank capture of the RCCL calls is supported but has only
            # been exercised on the driver's multi-GPU node; the replay buys
            # < 1 % at these kernel times, so it is opt-in there)
            mode = os.environ.get("BDX_GRAPH", "1")
            use_graph = mode == "2" or (mode == "1" and comm.size == 1)
        t = op.t
        self._latd = np.ascontiguousarray(pb.latd, dtype=np.int64)
        self._own = np.array(pb.lat.owned_hi, dtype=np.int64)
        self._ip = np.array([op.version, op.affine_code, pb.degree, t.nq, op.nblocks, op.nty,
                             op.ntz, op.sy, op.sz, int(use_graph)], dtype=np.int32)
        self._wts = np.ascontiguousarray(t.wts, dtype=np.float64)
        self._qpts = np.ascontiguousarray(t.qpts, dtype=np.float64)
        self.upart = torch.zeros(self.lib.bdx_hip_partials_size(), dtype=torch.float64,
                                 device=pb.device)
        fo, gh = halo.owned_faces, halo.ghosts
        bufs = [cg.x, cg.r, op.p_old, op.p_new, cg.y, op.yb, op.zb, op.cb, pb.xv, cg.scal,
                op.partials, self.upart, halo.buf_a, halo.buf_b, fo.table, gh.table, pb.kc]
        self._keep = bufs
        self._ptrs = (ctypes.c_void_p * len(bufs))(*[ptr(b) for b in bufs])
        self._hs = np.array([len(fo.boxes), fo.total, len(gh.boxes), gh.total], dtype=np.int64)
        self._fc = np.array(fo.counts, dtype=np.int64)
        self._gc = np.array(gh.counts, dtype=np.int64)
        uid = (ctypes.c_char * 128)()
        self.group = 0
        if comm.size == 1:
            transport = 0
        elif hasattr(comm, "g"):  # ThreadComm: ranks are threads of this process
            transport = 2
            self.group = id(comm.g)
        elif comm.backend == "nccl":
            transport = 1
            if comm.rank == 0:
                n = self.lib.bdx_rt_nccl_unique_id(uid)
                if n <= 0:
                    raise RuntimeError("ncclGetUniqueId failed")
            ids = comm.gather_objects(bytes(uid) if comm.rank == 0 else None)
            ctypes.memmove(uid, ids[0], 128)
        else:
            raise RuntimeError(f"native CG runtime: no transport for backend {comm.backend!r}")
        self.transport = ("none", "rccl", "thread")[transport]
        self.h = self.lib.bdx_rt_create(
            int(pb.dtype == torch.float64), ptr(self._latd), ptr(self._own), ptr(self._ip),
            float(pb.kappa), ptr(self._wts), ptr(self._qpts), ptr(op.tabs), self._ptrs,
            ptr(self._hs), ptr(self._fc), ptr(self._gc), transport, comm.size, comm.rank, uid,
            self.group, _stream())
        if not self.h:
            raise RuntimeError("bdx_rt_create failed (unsupported kernel or RCCL init error)")

    def reset(self) -> None:
        _check(self.lib.bdx_rt_reset(self.h), "rt_reset")

    def iterate(self, n: int) -> None:
        _check(self.lib.bdx_rt_iterate(self.h, int(n)), "rt_iterate")
        it, graphs = ctypes.c_long(0), ctypes.c_int(0)
        self.lib.bdx_rt_state(self.h, ctypes.byref(it), ctypes.byref(graphs))
        self.cg.it = it.value
        self.graphs = bool(graphs.value)

    def close(self) -> None:
        if getattr(self, "h", None):
            torch.cuda.synchronize()
            self.lib.bdx_rt_destroy(self.h)
            self.h = None
            if self.group:
                self.lib.bdx_rt_release_group(self.group)

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass
