"""EmulatedRankComm (parallel/comm.py) and scripts/emulate_rank.py on the CPU.

The emulated rank is how profiles/r5_split_schedule.md times one rank of an
N-rank run on a single GPU, so its problem must be exactly that rank's block:
the owned box, the ghost planes and the halo boxes of the same rank in a real
N-rank run (here: ThreadComm ranks, run_threaded).
"""

import os
import sys

import torch

from benchmark_dolfinx_amd.models.poisson import PoissonProblem
from benchmark_dolfinx_amd.parallel.comm import EmulatedRankComm, run_threaded

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _block(pb):
    lat = pb.lat
    return {
        "pgrid": tuple(lat.pgrid),
        "owned_hi": tuple(lat.owned_hi),
        "gh": tuple(lat.gh),
        "latd": tuple(int(v) for v in pb.latd),
        "send": [(tuple(b.lo), tuple(b.hi)) for b in lat.halo_send_boxes()],
        "recv": [(tuple(b.lo), tuple(b.hi)) for b in lat.halo_recv_boxes()],
        "ndofs_global": pb.ndofs_global,
    }


def test_emulated_collectives_are_local():
    c = EmulatedRankComm(3, 8)
    assert (c.rank, c.size, c.backend) == (3, 8, "emulated")
    assert c.allreduce_scalar(2.5, "sum") == 2.5
    assert c.allreduce_scalar(2.5, "max") == 2.5
    out = torch.ones(6)
    c.alltoallv(out, torch.arange(6.0), [1] * 6, [1] * 6)
    assert torch.equal(out, torch.zeros(6))
    assert c.gather_objects("x") == ["x"] * 8
    assert c.barrier() is None


def test_emulated_rank_block_matches_the_real_rank():
    nranks, nx, P = 4, (6, 7, 9), 2
    real = run_threaded(nranks, lambda comm: _block(
        PoissonProblem(comm, nx, P, 1, False, torch.float64, "cpu", 0.0)))
    for r in range(nranks):
        pb = PoissonProblem(EmulatedRankComm(r, nranks), nx, P, 1, False, torch.float64, "cpu", 0.0)
        assert _block(pb) == real[r], r


def test_pick_rank_prefers_y_and_z_ghosts():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import emulate_rank
    from benchmark_dolfinx_amd.fem.mesh import make_local_lattice
    nx = (40, 44, 48)
    for nranks in (2, 4, 8):
        lats = [make_local_lattice(r, nranks, nx, 3, whole_x=True) for r in range(nranks)]
        r = emulate_rank.pick_rank(nranks, nx, 3)
        both = [q for q, lat in enumerate(lats) if lat.gh[1] and lat.gh[2]]
        if both:  # the split schedule's two boundary launches exist on that rank
            assert r in both, (nranks, r, both)
        halo = [max(sum(b.size for b in lat.halo_send_boxes()),
                    sum(b.size for b in lat.halo_recv_boxes())) for lat in lats]
        pool = both or list(range(nranks))
        assert halo[r] == max(halo[q] for q in pool)
