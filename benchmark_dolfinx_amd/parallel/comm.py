"""Process-group plumbing: one process per GPU over torch.distributed.

The reference is SPMD over GPU-aware MPI with an external `select_gpu`
wrapper for device binding (README.md:94-104, quirk Q13).  Here:

* ranks come from the torchrun environment (RANK / WORLD_SIZE /
  LOCAL_RANK / MASTER_ADDR / MASTER_PORT), the device is bound from
  LOCAL_RANK before the process group is created;
* backend ``nccl`` (= RCCL on ROCm, over xGMI intra-node) for the GPU
  platform, ``gloo`` for the CPU platform (multi-process CPU tests);
* every collective works on tensors resident where the data lives: CG dot
  products are all-reduced as float64 *device* scalars (no host round trip,
  unlike the host-scalar MPI_Allreduce of src/cg.hpp:76); halo traffic is
  one all-to-all(v) per exchange (parallel/halo.py).
"""

from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


class Comm:
    """Thin wrapper; a size-1 Comm makes every collective a no-op."""

    def __init__(self):
        self.enabled = dist.is_available() and dist.is_initialized()
        self.rank = dist.get_rank() if self.enabled else 0
        self.size = dist.get_world_size() if self.enabled else 1
        self.backend = dist.get_backend() if self.enabled else "none"

    # ----------------------------------------------------------- collectives
    def allreduce_(self, t: torch.Tensor, op: str = "sum", async_op: bool = False):
        if self.size == 1:
            return None
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN}[op]
        return dist.all_reduce(t, op=rop, async_op=async_op)

    @property
    def device(self) -> torch.device:
        """Where this backend's collectives take tensors (RCCL: the GPU only)."""
        if self.backend == "nccl":
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def allreduce_scalar(self, v: float, op: str = "sum") -> float:
        if self.size == 1:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.device)
        self.allreduce_(t, op)
        return float(t.item())

    def alltoallv(self, out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits,
                  async_op: bool = False):
        if self.size == 1:
            return None
        return dist.all_to_all_single(out, inp, list(out_splits), list(in_splits),
                                      async_op=async_op)

    def barrier(self):
        if self.size > 1:
            if self.backend == "nccl":
                dist.barrier(device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier()

    def gather_objects(self, obj):
        if self.size == 1:
            return [obj]
        out = [None] * self.size
        dist.all_gather_object(out, obj)
        return out


class _Done:
    def wait(self):
        return None


class ThreadGroup:
    """Shared state of an in-process group of ranks (one Python thread each)."""

    _serial = iter(range(1, 1 << 62))  # process-unique group ids (id() gets reused)

    def __init__(self, size: int):
        import threading
        self.uid = next(ThreadGroup._serial)
        self.size = size
        self.barrier = threading.Barrier(size)
        self.slots = [None] * size


class ThreadComm(Comm):
    """Rank of an in-process thread group.

    Lets tests (and rehearsals) run R ranks of the real code path in one
    process -- on the CPU, or on ONE GPU with the HIP kernels (RCCL cannot put
    two ranks on one device).  Collectives are executed with tensor copies on
    the device's default stream, ordered by the group barrier; reductions sum
    in rank order, so results are deterministic.
    """

    def __init__(self, group: ThreadGroup, rank: int, emulate: str = "thread"):
        self.enabled = True
        self.rank = rank
        self.size = group.size
        # emulate="nccl": reject host tensors in collectives like RCCL does, so
        # single-GPU tests catch host-scalar collectives in GPU code paths
        self.backend = emulate
        self.g = group

    def _check_dev(self, t):
        if self.backend == "nccl" and isinstance(t, torch.Tensor) and not t.is_cuda:
            raise RuntimeError("RCCL collectives take device tensors only (got a host tensor)")

    def _sync_dev(self, t):
        if isinstance(t, torch.Tensor) and t.is_cuda:
            torch.cuda.synchronize(t.device)

    def allreduce_(self, t, op: str = "sum", async_op: bool = False):
        self._check_dev(t)
        if self.size == 1:
            return _Done() if async_op else None
        self.g.slots[self.rank] = t.detach().clone()
        self._sync_dev(t)
        self.g.barrier.wait()
        vals = [s.to(t.device) for s in self.g.slots]
        acc = vals[0].clone()
        for v in vals[1:]:
            if op == "sum":
                acc += v
            elif op == "max":
                acc = torch.maximum(acc, v)
            else:
                acc = torch.minimum(acc, v)
        self._sync_dev(acc)
        self.g.barrier.wait()
        t.copy_(acc)
        self._sync_dev(t)
        return _Done() if async_op else None

    def alltoallv(self, out, inp, out_splits, in_splits, async_op: bool = False):
        self._check_dev(out)
        self._check_dev(inp)
        if self.size == 1:
            return _Done() if async_op else None
        self._sync_dev(inp)
        self.g.slots[self.rank] = (inp, list(in_splits))
        self.g.barrier.wait()
        off_out = 0
        for p in range(self.size):
            pin, psplits = self.g.slots[p]
            n = psplits[self.rank]
            assert n == out_splits[p], (n, out_splits[p])
            if n:
                o = sum(psplits[: self.rank])
                out[off_out: off_out + n].copy_(pin[o: o + n].to(out.device))
            off_out += out_splits[p]
        self._sync_dev(out)
        self.g.barrier.wait()
        return _Done() if async_op else None

    def barrier(self):
        self.g.barrier.wait()

    def gather_objects(self, obj):
        self.g.slots[self.rank] = obj
        self.g.barrier.wait()
        out = list(self.g.slots)
        self.g.barrier.wait()
        return out


class EmulatedRankComm(Comm):
    """Rank `rank` of an N-rank run, alone on this device (experiments:
    scripts/emulate_rank.py).

    The problem is that rank's block of the N-rank partition, ghost planes
    included, so the operator and the native runtime's split schedule run
    exactly as on the rank of a real N-GPU run; the native runtime replaces
    RCCL by modelled link times (runtime.hip LinkEmuTransport).  Host-side
    collectives are local no-ops: all-reduces return the rank's own values
    and all-to-alls deliver zeros, so norms are this rank's, not the global
    problem's -- for timing the schedule, not for results.
    """

    def __init__(self, rank: int, size: int):
        self.enabled = True
        self.rank = rank
        self.size = size
        self.backend = "emulated"

    @property
    def device(self) -> torch.device:
        if torch.cuda.is_available():
            return torch.device("cuda", torch.cuda.current_device())
        return torch.device("cpu")

    def allreduce_(self, t, op: str = "sum", async_op: bool = False):
        return _Done() if async_op else None

    def allreduce_scalar(self, v: float, op: str = "sum") -> float:
        return float(v)

    def alltoallv(self, out, inp, out_splits, in_splits, async_op: bool = False):
        out.zero_()
        return _Done() if async_op else None

    def barrier(self):
        return None

    def gather_objects(self, obj):
        return [obj] * self.size


def run_threaded(size: int, fn, *args, emulate: str = "thread", **kwargs):
    """Run fn(comm, *args) on `size` in-process ranks; returns the per-rank results."""
    import threading
    group = ThreadGroup(size)
    results = [None] * size
    errors = []

    def body(r):
        try:
            if torch.cuda.is_available():
                torch.cuda.set_device(0)
            results[r] = fn(ThreadComm(group, r, emulate), *args, **kwargs)
        except BaseException as e:  # pragma: no cover - re-raised below
            errors.append(e)
            group.barrier.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(size)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errors:
        raise errors[0]
    return results


def init_distributed(platform: str = "gpu", timeout_s: float = 600.0) -> Comm:
    """Initialise the process group from the torchrun environment (if any)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if platform == "gpu" and torch.cuda.is_available():
        torch.cuda.set_device(local_rank)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        backend = "nccl" if platform == "gpu" else "gloo"
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local_rank)
        dist.init_process_group(**kw)
    return Comm()


def finalize() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
