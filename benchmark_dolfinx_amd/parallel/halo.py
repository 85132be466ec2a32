"""Plane-halo exchange over all-to-all(v) (RCCL on GPU, gloo on CPU).

Replaces the DOLFINx `Scatterer` + the repo's pack/unpack kernels
(`src/vector.hpp:31-149`, call sites `src/laplacian.hpp:286-320`,
`src/cg.hpp:133-136`).  With the analytic partition of fem/mesh.py every
message is a box of the local lattice:

* forward (owner -> ghost): each rank sends the lower faces of its owned box
  (plane index 0 in the split axes) to its <= 7 lower neighbours and receives
  its ghost planes (index L-1) from its <= 7 upper neighbours;
* reverse (ghost partial sums -> owner, add): the same boxes with the roles
  swapped.

One all-to-all(v) per exchange; the split sizes are zero for non-neighbours.
On a 2x2x2 split of 8 MI355X each rank talks to at most 7 peers, i.e. one
message per xGMI link.  Unlike the reference (quirk Q1: one 512-thread block
unpacks only the first 512 ghosts inside apply) every ghost is unpacked.
"""

from __future__ import annotations

import numpy as np
import torch

from ..fem.mesh import HaloBox, LocalLattice
from .comm import Comm


class _Side:
    """Boxes for one direction of one exchange, ordered by peer rank."""

    def __init__(self, boxes: list[HaloBox], nranks: int, lat: LocalLattice, device):
        self.boxes = sorted(boxes, key=lambda b: b.peer)
        self.counts = [0] * nranks
        for b in self.boxes:
            self.counts[b.peer] += b.size
        self.total = sum(self.counts)
        tab = []
        off = 0
        for b in self.boxes:
            e = [h - l for l, h in zip(b.lo, b.hi)]
            tab.append(list(b.lo) + e + [off])
            off += b.size
        self.table = torch.tensor(np.array(tab, dtype=np.int64).reshape(-1, 7),
                                  device=device)
        # flat indices (CPU path and tests)
        idx = []
        L1, ld = lat.L[1], lat.ld
        for b in self.boxes:
            i = np.arange(b.lo[0], b.hi[0])[:, None, None]
            j = np.arange(b.lo[1], b.hi[1])[None, :, None]
            k = np.arange(b.lo[2], b.hi[2])[None, None, :]
            idx.append(((i * L1 + j) * ld + k).ravel())
        flat = np.concatenate(idx) if idx else np.zeros(0, dtype=np.int64)
        self.index = torch.from_numpy(flat.astype(np.int64)).to(device)


class HaloExchange:
    def __init__(self, lat: LocalLattice, comm: Comm, dtype, device, kernels=None):
        self.lat = lat
        self.comm = comm
        self.device = torch.device(device)
        self.kernels = kernels  # ops.kernels.HipKernels on GPU, None on CPU
        self.owned_faces = _Side(lat.halo_send_boxes(), comm.size, lat, device)
        self.ghosts = _Side(lat.halo_recv_boxes(), comm.size, lat, device)
        n = max(self.owned_faces.total, self.ghosts.total, 1)
        self.buf_a = torch.empty(n, dtype=dtype, device=device)
        self.buf_b = torch.empty(n, dtype=dtype, device=device)
        self.active = comm.size > 1 and (self.owned_faces.total + self.ghosts.total) > 0

    @property
    def bytes_per_exchange(self) -> int:
        return max(self.owned_faces.total, self.ghosts.total) * self.buf_a.element_size()

    # ------------------------------------------------------------- kernels
    def _pack(self, x: torch.Tensor, side: _Side, buf: torch.Tensor):
        if side.total == 0:
            return
        if self.kernels is not None:
            self.kernels.box_copy(0, x, self.lat, side, buf)
        else:
            torch.index_select(x.view(-1), 0, side.index, out=buf[: side.total])

    def _unpack(self, x: torch.Tensor, side: _Side, buf: torch.Tensor, add: bool):
        if side.total == 0:
            return
        if self.kernels is not None:
            self.kernels.box_copy(2 if add else 1, x, self.lat, side, buf)
        elif add:
            x.view(-1).index_add_(0, side.index, buf[: side.total])
        else:
            x.view(-1).index_copy_(0, side.index, buf[: side.total])

    # ------------------------------------------------------------ exchanges
    def forward_begin(self, x: torch.Tensor):
        """Pack owned lower faces and post the all-to-all (async)."""
        if not self.active:
            return None
        self._pack(x, self.owned_faces, self.buf_a)
        return self.comm.alltoallv(self.buf_b[: self.ghosts.total],
                                   self.buf_a[: self.owned_faces.total],
                                   self.ghosts.counts, self.owned_faces.counts,
                                   async_op=True)

    def forward_end(self, x: torch.Tensor, work) -> None:
        if not self.active:
            return
        if work is not None:
            work.wait()
        self._unpack(x, self.ghosts, self.buf_b, add=False)

    def forward(self, x: torch.Tensor) -> None:
        self.forward_end(x, self.forward_begin(x))

    def reverse_begin(self, y: torch.Tensor):
        """Pack ghost-plane partial sums and post the all-to-all (async)."""
        if not self.active:
            return None
        self._pack(y, self.ghosts, self.buf_a)
        return self.comm.alltoallv(self.buf_b[: self.owned_faces.total],
                                   self.buf_a[: self.ghosts.total],
                                   self.owned_faces.counts, self.ghosts.counts,
                                   async_op=True)

    def reverse_end(self, y: torch.Tensor, work) -> None:
        if not self.active:
            return
        if work is not None:
            work.wait()
        self._unpack(y, self.owned_faces, self.buf_b, add=True)

    def reverse(self, y: torch.Tensor) -> None:
        self.reverse_end(y, self.reverse_begin(y))
