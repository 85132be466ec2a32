"""Python handle of the native C++ CG runtime (csrc/hip/runtime.hip).

After the CG prologue (r0 = b - A x0, rho0 = r0.r0; FusedLaplacianGPU.cg_start)
the whole iteration loop -- halo exchange, fused operator, reductions,
all-reduces, r/x updates -- runs in C++ on the current HIP stream, with the
steady-state iterations replayed from hipGraphs.  Transport:

* ``rccl``   one process per GPU (torchrun or bench.py's own launcher); the
  runtime opens its own RCCL communicator, bootstrapped by exchanging an
  ncclUniqueId over the existing torch.distributed group, and exchanges halos
  with grouped ncclSend/ncclRecv to the neighbours only, on a second stream
  overlapped with the interior tiles of the operator;
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


PHASES = ("halo_fwd", "op_interior", "op_boundary", "halo_rev", "join_rev_add",
          "reduce_allreduce_pap", "update_rr", "allreduce_rr", "iteration",
          # offsets from the iteration start: the comm-stream chain (forward
          # exchange, boundary tiles, reverse send) is hidden when it ends
          # before the interior tiles on the compute stream do
          "t_halo_fwd_done", "t_boundary_done", "t_halo_rev_done",
          "t_op_interior_done")


def _agree(comm, ok: bool) -> bool:
    """True iff every rank reports ok (a MIN all-reduce over the torch group)."""
    if comm.size == 1:
        return ok
    return comm.allreduce_scalar(1.0 if ok else 0.0, "min") > 0.5


class NativeCGRuntime:
    """Handle of one rank's native CG loop.

    Construction is collective and all-or-nothing: every rank first builds
    its runtime locally (no communication), the ranks agree that all
    succeeded, then the RCCL communicator is opened (bounded by the
    watchdog deadline) and the ranks agree again.  If any rank fails at
    either step every rank releases its handle and raises
    NativeRuntimeUnavailable, so all ranks take the same fallback (a rank
    on native RCCL calls and a rank on torch collectives would never match).
    """

    # test hook: rank whose local creation is made to fail
    _inject_fail_rank: int | None = None

    def __init__(self, op, cg, use_graph: bool | None = None, overlap: bool | None = None):
        pb = op.pb
        self.op, self.cg, self.pb = op, cg, pb
        self.lib = native.hip()
        self.h = None
        comm = pb.comm
        halo = pb.halo
        if use_graph is None:
            # BDX_GRAPH=0 (default) eager launches at every rank count, 1 graph
            # replay on a single rank, 2 also with RCCL (the two-stream
            # fork/join iteration captures RCCL calls).  One launch mode for
            # every N keeps the weak-scaling points comparable; at N = 1 graph
            # replay and eager launches measured equal (60.12 vs 60.17 GDoF/s
            # same box, profiles/r3_graph_ab.md): the host runs far ahead of
            # a 5 ms iteration, so launch overhead is hidden either way.
            mode = os.environ.get("BDX_GRAPH", "0")
            use_graph = mode == "2" or (mode == "1" and comm.size == 1)
        if overlap is None:
            overlap = os.environ.get("BDX_OVERLAP", "1") != "0"
        self.kind = "dofmap" if getattr(op, "name", "") == "dofmap" else "fused"
        self.group = 0
        if comm.size == 1:
            transport = 0
        elif hasattr(comm, "g"):  # ThreadComm: ranks are threads of this process
            transport = 2
            self.group = comm.g.uid  # unique per group: a reused id() could
            # pick up a stale group of a runtime that was not closed yet
        elif comm.backend == "nccl":
            transport = 1
        elif comm.backend == "emulated":  # EmulatedRankComm: modelled links
            transport = 3
            halo.buf_a.zero_()  # the emulated copies move finite data only
            halo.buf_b.zero_()
        else:
            transport = -1
        self.transport = {0: "none", 1: "rccl", 2: "thread", 3: "emulated"}.get(
            transport, "unsupported")
        self.upart = torch.zeros(self.lib.bdx_hip_partials_size(), dtype=torch.float64,
                                 device=pb.device)
        self.x = cg.x
        fo, gh = halo.owned_faces, halo.ghosts
        self._hs = np.array([len(fo.boxes), fo.total, len(gh.boxes), gh.total], dtype=np.int64)
        self._fc = np.array(fo.counts, dtype=np.int64)
        self._gc = np.array(gh.counts, dtype=np.int64)
        self._latd = np.ascontiguousarray(pb.latd, dtype=np.int64)
        ok = transport >= 0 and comm.rank != self._inject_fail_rank
        if self.kind == "dofmap":
            ok = ok and self._create_dofmap(op, cg, use_graph, overlap, transport)
        else:
            ok = ok and self._create_fused(op, cg, use_graph, overlap, transport)
        self._connect(comm, ok, transport)

    def _create_dofmap(self, op, cg, use_graph, overlap, transport) -> bool:
        """The dofmap data model's loop (runtime.hip DofCGRuntime)."""
        pb, halo = self.pb, self.pb.halo
        self.tiled = False
        self._ip = np.array([pb.degree, pb.tables.nq, op.geom, int(op.inner.numel()),
                             int(op.outer.numel()), int(use_graph), int(overlap)], dtype=np.int32)
        bufs = [cg.x, cg.r, op.p_a, op.p_b, cg.y, cg.scal, cg.partials, self.upart,
                halo.buf_a, halo.buf_b, halo.owned_faces.table, halo.ghosts.table, op.tab,
                op.inner, op.outer, op.cdofs, op.cverts, op.coords, op.flags, op.G, op.kc]
        self._keep = bufs
        self._ptrs = (ctypes.c_void_p * len(bufs))(*[ptr(b) for b in bufs])
        self.h = self.lib.bdx_rt_create_dofmap(
            int(pb.dtype == torch.float64), ptr(self._latd), ptr(self._ip), int(cg.r.numel()),
            float(pb.kappa), self._ptrs, ptr(self._hs), ptr(self._fc), ptr(self._gc), transport,
            pb.comm.size, pb.comm.rank, self.group, _stream())
        return bool(self.h)

    def _create_fused(self, op, cg, use_graph, overlap, transport) -> bool:
        pb, halo = self.pb, self.pb.halo
        t = op.t
        self._own = np.array(pb.lat.owned_hi, dtype=np.int64)
        self._ip = np.array([op.version, op.affine_code, pb.degree, t.nq, op.nblocks, op.nty,
                             op.ntz, op.sy, op.sz, int(use_graph), int(overlap), op.nseg],
                            dtype=np.int32)
        self._wts = np.ascontiguousarray(t.wts, dtype=np.float64)
        self._qpts = np.ascontiguousarray(t.qpts, dtype=np.float64)
        fo, gh = halo.owned_faces, halo.ghosts
        # Tiled vector storage for the x-march kernels: each (y, z) tile's
        # patch of an x-plane is contiguous, so the kernels' writes are whole
        # lines (profiles/r2_march_bw.md).  BDX_TILED=0: the lattice layout;
        # 1 (default): fused5 and fused3's x-trilinear instance
        # (perturbed Q3 +2 %, Q6 +3 %, Q6 FP32 +5 %, profiles/r2_xtrilinear.md);
        # 2: every fused3 instance (the general-geometry kernel is
        # compute-bound: Q3 +0.6 %, Q6 -2.4 % on tiled storage,
        # profiles/r2_launder.md).  The tiled r update needs 16-byte tile
        # planes.
        mode = os.environ.get("BDX_TILED", "1")
        esz = 8 if pb.dtype == torch.float64 else 4
        f3 = op.version == 3 and (mode == "2" or getattr(op, "x_trilinear", False))
        self.tiled = (mode != "0" and (op.version == 5 or f3)
                      and (op.sy * op.sz * esz) % 16 == 0)
        self._latdT = None
        self._tbufs = []
        if self.tiled:
            self._latdT = np.ascontiguousarray(pb.lat.as_int64((op.sy, op.sz)), dtype=np.int64)
            n = pb.lat.tiled_size(op.sy, op.sz)
            self._tbufs = [torch.zeros(n, dtype=pb.dtype, device=pb.device) for _ in range(5)]
        self._tptrs = (ctypes.c_void_p * 5)(*[ptr(b) for b in self._tbufs]) if self.tiled else None
        bufs = [cg.x, cg.r, op.p_old, op.p_new, cg.y, op.yb, op.zb, op.cb, pb.xv, cg.scal,
                op.partials, self.upart, halo.buf_a, halo.buf_b, fo.table, gh.table, pb.kc]
        self._keep = bufs + [op.tabs]
        self._ptrs = (ctypes.c_void_p * len(bufs))(*[ptr(b) for b in bufs])
        del fo, gh
        self.h = self.lib.bdx_rt_create(
            int(pb.dtype == torch.float64), ptr(self._latd), ptr(self._own), ptr(self._ip),
            float(pb.kappa), ptr(self._wts), ptr(self._qpts), ptr(op.tabs), self._ptrs,
            ptr(self._hs), ptr(self._fc), ptr(self._gc), transport, pb.comm.size, pb.comm.rank,
            self.group, _stream(), ptr(self._latdT), self._tptrs)
        return bool(self.h)

    def _connect(self, comm, ok: bool, transport: int) -> None:
        """1) every rank created its runtime locally (no communication): agree;
        2) open the RCCL communicator (ncclUniqueId from rank 0 over the torch
        group), bounded by the watchdog deadline: agree again."""
        if not _agree(comm, ok):
            self.close()
            raise NativeRuntimeUnavailable(
                "bdx_rt_create failed on at least one rank (unsupported kernel, no transport "
                f"for backend {comm.backend!r}, or an injected failure)")
        # 2) open the runtime's own RCCL communicator (ncclUniqueId from rank 0
        #    over the torch group); bounded by the watchdog deadline
        if transport == 1:
            uid = (ctypes.c_char * 128)()
            good = True
            if comm.rank == 0:
                good = self.lib.bdx_rt_nccl_unique_id(uid) > 0
            ids = comm.gather_objects(bytes(uid) if (comm.rank == 0 and good) else None)
            if ids[0] is None:
                self.close()
                raise NativeRuntimeUnavailable("ncclGetUniqueId failed on rank 0")
            ctypes.memmove(uid, ids[0], 128)
            ok = self.lib.bdx_rt_connect(self.h, uid, comm.rank) == 0
            if not _agree(comm, ok):
                self.close()
                raise NativeRuntimeUnavailable("ncclCommInitRank failed on at least one rank")
        self.overlap = bool(self.lib.bdx_rt_overlap(self.h))
        self.tiled = bool(self.lib.bdx_rt_tiled(self.h))
        self.graphs = False

    def comm_priority(self) -> dict:
        """Priority of the comm stream and the device's range (HIP: a lower
        value is a higher priority)."""
        out = (ctypes.c_int * 3)()
        _check(self.lib.bdx_rt_comm_priority(self.h, out), "rt_comm_priority")
        return {"least": out[0], "greatest": out[1], "comm_stream": out[2]}

    def preflight(self, timeout_s: float = 60.0) -> dict:
        """One forward halo exchange and a device all-reduce of (rank + 1),
        bounded by `timeout_s`: raises if a peer never joins or the sum is
        wrong (every rank must call it)."""
        out = (ctypes.c_double * 2)()
        _check(self.lib.bdx_rt_preflight(self.h, float(timeout_s), out), "rt_preflight")
        n = self.pb.comm.size
        want = n * (n + 1) / 2
        if out[1] != want:
            raise RuntimeError(f"pre-flight all-reduce returned {out[1]}, expected {want}")
        return {"ms": float(out[0]), "allreduce": float(out[1])}

    def overlap_probe(self, n: int, reps: int = 5) -> dict:
        """One-rank probe of the split schedule (runtime.hip overlap_probe):
        an RCCL self send/recv of n doubles, the boundary tiles and a second
        send/recv on the comm stream under the interior tiles.  Clobbers the
        CG state (restart CG afterwards)."""
        buf = torch.zeros(2 * int(n), dtype=torch.float64, device=self.pb.device)
        buf[:n] = torch.arange(n, dtype=torch.float64, device=self.pb.device)
        out = (ctypes.c_double * 6)()
        torch.cuda.synchronize()
        _check(self.lib.bdx_rt_overlap_probe(self.h, int(n), ptr(buf), int(reps), out),
               "rt_overlap_probe")
        torch.cuda.synchronize()
        ok = bool(torch.equal(buf[n:], buf[:n]))
        keys = ("chain_alone_ms", "interior_alone_ms", "chain_done_ms", "interior_done_ms",
                "exchange_alone_ms", "fwd_exchange_done_ms")
        rec = {k: float(v) for k, v in zip(keys, out)}
        rec["exchange_ok"] = ok
        rec["bytes"] = int(n) * 8
        return rec

    def comm_ranks(self) -> int:
        """Ranks of the runtime's own communicator (ncclCommCount for RCCL)."""
        return int(self.lib.bdx_rt_comm_count(self.h))

    def bind_x(self, x: torch.Tensor) -> None:
        """Point the runtime at a new iterate (drops the captured graphs)."""
        if x.data_ptr() != self.x.data_ptr():
            _check(self.lib.bdx_rt_bind_x(self.h, ptr(x)), "rt_bind_x")
            self.x = x
            self._keep[0] = x

    def reset(self) -> None:
        _check(self.lib.bdx_rt_reset(self.h), "rt_reset")

    def _sync_state(self) -> None:
        it, graphs = ctypes.c_long(0), ctypes.c_int(0)
        self.lib.bdx_rt_state(self.h, ctypes.byref(it), ctypes.byref(graphs))
        self.cg.it = it.value
        self.graphs = bool(graphs.value)

    def iterate(self, n: int) -> None:
        _check(self.lib.bdx_rt_iterate(self.h, int(n)), "rt_iterate")
        self._sync_state()

    def iterate_timed(self, n: int) -> list[float]:
        """iterate(n) and return the device time (ms) of each step, from
        timing events recorded between the steps (waits for the steps)."""
        out = (ctypes.c_float * max(1, int(n)))()
        _check(self.lib.bdx_rt_iterate_timed(self.h, int(n), out), "rt_iterate_timed")
        self._sync_state()
        return [float(v) for v in out[:int(n)]]

    def wait(self) -> None:
        """Host wait for the queued iterations, bounded by the RCCL deadline
        (BDX_RCCL_TIMEOUT_S): a hung peer raises instead of blocking forever."""
        _check(self.lib.bdx_rt_wait(self.h), "rt_wait")

    def profile(self, n: int) -> dict:
        """n eager iterations with hipEvent phase timers -> mean ms per phase."""
        out = (ctypes.c_double * len(PHASES))()
        _check(self.lib.bdx_rt_profile(self.h, int(n), out, len(PHASES)), "rt_profile")
        self._sync_state()
        ph = {k: float(v) for k, v in zip(PHASES, out)}
        # meaningful only for the split (two-stream) schedule
        split = self.overlap
        ph["halo_fwd_hidden"] = (ph["t_halo_fwd_done"] <= ph["t_op_interior_done"]) if split else None
        ph["halo_rev_hidden"] = (ph["t_halo_rev_done"] <= ph["t_op_interior_done"]) if split else None
        return ph

    def close(self) -> None:
        if getattr(self, "h", None):
            # bounded by the RCCL deadline (a hung peer must not block the
            # teardown forever), then the device for the caller's stream
            rc = self.lib.bdx_rt_wait(self.h)
            if rc == 0:
                torch.cuda.synchronize()
            self.lib.bdx_rt_destroy(self.h)
            self.h = None
        if getattr(self, "group", 0):
            self.lib.bdx_rt_release_group(self.group)
            self.group = 0

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass


class NativeRuntimeUnavailable(RuntimeError):
    """Raised on every rank when the native runtime cannot run on all ranks."""
