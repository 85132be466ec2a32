"""Unpreconditioned conjugate gradients (reference: `cg_solve`, src/cg.hpp:89-169).

Two implementations with the reference's algorithm (x0 given, r0 = b - A x0,
p0 = r0, rtol = 0 runs exactly max_iter iterations):

* `cg_solve`: generic, host scalars (used by the CPU platform and the CSR
  comparison path).
* `cg_solve_device`: GPU, every scalar stays on the device.  Per iteration:
  apply (+ halo), dot(p, y) -> all-reduce, fused {x += a p; r -= a y;
  r.r} -> all-reduce, p = b p + r.  alpha/beta are formed inside the kernels
  from float64 device slots, ping-ponging the r.r slot between iterations
  so no kernel reads a slot another kernel of the same iteration writes.
  One halo exchange per iteration (the reference does two, quirk Q2) and no
  host synchronisation (quirk Q3).

When the operator provides `cg_start` / `cg_iterate` (the fused structured
kernel, models/fused.py) the device loop delegates to it.
"""

from __future__ import annotations

import torch


def cg_solve(op, pb, x: torch.Tensor, b: torch.Tensor, max_iter: int,
             rtol: float = 0.0) -> int:
    r = pb.new_vector()
    y = pb.new_vector()
    op.apply(x, y)
    r.copy_(b - y)
    p = r.clone()
    rnorm0 = pb.inner(p, r)
    rnorm = rnorm0
    rtol2 = rtol * rtol
    k = 0
    while k < max_iter:
        k += 1
        op.apply(p, y)
        alpha = rnorm / pb.inner(p, y)
        x.add_(p, alpha=alpha)
        r.add_(y, alpha=-alpha)
        rnorm_new = pb.inner(r, r)
        beta = rnorm_new / rnorm
        rnorm = rnorm_new
        if rnorm0 > 0 and rnorm / rnorm0 < rtol2:
            break
        p.mul_(beta).add_(r)
    return k


class DeviceCG:
    """Device-resident CG state for the GPU platform."""

    # float64 scalar slots
    RR0, RR1, PAP = 0, 1, 2

    def __init__(self, pb):
        self.pb = pb
        self.k = pb.kernels
        dev = pb.device
        self.scal = torch.zeros(8, dtype=torch.float64, device=dev)
        self.partials = torch.zeros(self.k.npart, dtype=torch.float64, device=dev)
        self.r = pb.new_vector()
        self.y = pb.new_vector()
        self.p = pb.new_vector()

    def _allreduce(self, slot: int) -> None:
        if self.pb.comm.size > 1:
            self.pb.comm.allreduce_(self.scal[slot: slot + 1])

    def start(self, op, x: torch.Tensor, b: torch.Tensor) -> None:
        """r0 = b - A x0, p0 = r0, rho0 = p0.r0 (the prologue of src/cg.hpp:98-112)."""
        self.op, self.x, self.it = op, x, 0
        if hasattr(op, "cg_start"):
            op.cg_start(self, x, b)
            return
        k, r, y, p, scal = self.k, self.r, self.y, self.p, self.scal
        op.apply(x, y)
        k.axpy(r, -1.0, y, b)
        p.copy_(r)
        k.dot(p, r, self.partials, scal, self.RR0)
        self._allreduce(self.RR0)

    def iterate(self, n: int, flush: bool = True) -> None:
        """Run n CG iterations (state persists across calls).  A fused
        operator lags its x update by one iteration; `flush=False` leaves the
        last one pending for the next call (x is then one update behind)."""
        op, x = self.op, self.x
        if hasattr(op, "cg_iterate"):
            op.cg_iterate(self, n, flush=flush)
            return
        k, r, y, p, scal = self.k, self.r, self.y, self.p, self.scal
        for _ in range(n):
            cur = self.RR0 if self.it % 2 == 0 else self.RR1
            nxt = self.RR1 if self.it % 2 == 0 else self.RR0
            op.apply(p, y)
            k.dot(p, y, self.partials, scal, self.PAP)
            self._allreduce(self.PAP)
            k.cg_update(x, r, p, y, scal, cur, self.PAP, nxt, self.partials)
            self._allreduce(nxt)
            k.p_update(p, r, scal, nxt, cur)
            self.it += 1

    def iterate_timed(self, n: int) -> list[float]:
        """iterate(n) plus the device time (ms) of each step.  The native
        runtime records timing events between its steps (same launches as
        iterate); the Python loop records torch events around each step."""
        rt = getattr(self.op, "_rt", None)
        if rt is not None:
            return rt.iterate_timed(n)
        if self.pb.platform != "gpu":
            self.iterate(n)
            return []
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        ev[0].record()
        for i in range(n):
            # one x flush at the end of the timed window (inside the last
            # step), as the native runtime's iterate(n) does
            self.iterate(1, flush=i == n - 1)
            ev[i + 1].record()
        ev[n].synchronize()
        return [ev[i].elapsed_time(ev[i + 1]) for i in range(n)]

    def wait(self) -> None:
        """Host wait for the queued iterations.  With the native runtime the
        wait is bounded by the RCCL deadline (a hung peer raises instead of
        blocking torch.cuda.synchronize forever)."""
        rt = getattr(self.op, "_rt", None)
        if rt is not None:
            rt.wait()
        elif self.pb.platform == "gpu":
            torch.cuda.synchronize()

    def solve(self, op, x: torch.Tensor, b: torch.Tensor, max_iter: int) -> int:
        self.start(op, x, b)
        self.iterate(max_iter)
        return max_iter

    def residual_norm2(self) -> float:
        slot = self.RR0 if self.it % 2 == 0 else self.RR1
        return float(self.scal[slot].item())


def cg_solve_device(op, pb, x: torch.Tensor, b: torch.Tensor, max_iter: int) -> int:
    return DeviceCG(pb).solve(op, x, b, max_iter)
