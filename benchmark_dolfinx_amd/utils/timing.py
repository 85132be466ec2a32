"""Named wall-clock timers and the end-of-run timing table.

Equivalent of `dolfinx::common::Timer` scopes and `list_timings` (MPI_MAX
reduced table; src/main.cpp:314, output format examples/slurm.out:33-62).
Timers here are flushed when the scope exits (the reference's
"% Create matfree operator" is never flushed, quirk Q10).  Optional roctx
ranges mark the same scopes for rocprofv3 (--marker-trace) when
BDX_ROCTX=1.
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import OrderedDict

_registry: "OrderedDict[str, list[float]]" = OrderedDict()
_roctx = None


def _roctx_lib():
    global _roctx
    if _roctx is None:
        _roctx = False
        if os.environ.get("BDX_ROCTX", "0") == "1":
            for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    _roctx = lib
                    break
                except OSError:
                    continue
    return _roctx or None


@contextlib.contextmanager
def timed(name: str, sync=None):
    """Time a scope (optionally calling `sync()` before reading the clock)."""
    lib = _roctx_lib()
    if lib:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        if sync is not None:
            sync()
        dt = time.perf_counter() - t0
        if lib:
            lib.roctxRangePop()
        rec = _registry.setdefault(name, [0, 0.0, 0.0])
        rec[0] += 1
        rec[1] += dt
        rec[2] = max(rec[2], dt)


def add_time(name: str, dt: float, reps: int = 1) -> None:
    rec = _registry.setdefault(name, [0, 0.0, 0.0])
    rec[0] += reps
    rec[1] += dt
    rec[2] = max(rec[2], dt)


def reset() -> None:
    _registry.clear()


def timings() -> dict:
    return {k: dict(reps=v[0], total=v[1], max=v[2]) for k, v in _registry.items()}


def list_timings(comm=None) -> str:
    """Rank-MAX reduced table (like dolfinx::list_timings(comm, MPI_MAX))."""
    names = list(_registry.keys())
    if comm is not None and comm.size > 1:
        allnames = comm.gather_objects(names)
        names = sorted(set(n for ns in allnames for n in ns))
        rows = []
        for n in names:
            rec = _registry.get(n, [0, 0.0, 0.0])
            reps = comm.allreduce_scalar(rec[0], "max")
            tot = comm.allreduce_scalar(rec[1], "max")
            rows.append((n, int(reps), tot))
    else:
        rows = [(n, _registry[n][0], _registry[n][1]) for n in names]
    w = max([len(r[0]) for r in rows] + [30])
    out = [f"[MAX] Summary of timings (wall){'':>{max(0, w - 28)}} |  reps  wall avg  wall tot",
           "-" * (w + 34)]
    for n, reps, tot in rows:
        avg = tot / reps if reps else 0.0
        out.append(f"{n:<{w}} | {reps:6d} {avg:9.6f} {tot:9.6f}")
    return "\n".join(out)
