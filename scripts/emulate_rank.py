#!/usr/bin/env python3
"""One rank of the N-GPU weak-scaled run, alone on this GPU, with modelled links.

RCCL refuses two ranks on one device and this pool has one GPU per box, so
the N-rank split schedule (runtime.hip CGRuntime::step: forward exchange ->
boundary tiles -> ghost fold -> reverse send on the comm stream, interior
tiles on the compute stream) is timed here on the block one rank of the
N-rank run owns -- ghost planes, tile split and halo counts exactly as on
that rank -- with the native runtime's LinkEmuTransport in place of RCCL:
every exchange holds a few CUs for max_peer(bytes) / link GB/s + latency,
every all-reduce for a fixed time (BDX_EMU_LINK_GBPS, BDX_EMU_LINK_LAT_US,
BDX_EMU_ALLREDUCE_US).  The same rank's owned block is then run as a
1-rank problem (no halo, serial schedule) for the comparison.

Prints one JSON line per run.  Reference schedule: src/laplacian.hpp:281-349.

  python scripts/emulate_rank.py --ranks 8 --config q3 [--rank R] [--steps K]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402
from benchmark_dolfinx_amd.fem.mesh import compute_mesh_size, make_local_lattice  # noqa: E402


def pick_rank(nranks: int, nx, degree: int) -> int:
    """The rank with the most halo traffic among those with both a y and a z
    ghost plane (the split schedule's two boundary tile launches)."""
    best, best_r = (-1, -1), 0
    for r in range(nranks):
        lat = make_local_lattice(r, nranks, nx, degree, whole_x=True)
        send = sum(b.size for b in lat.halo_send_boxes())
        recv = sum(b.size for b in lat.halo_recv_boxes())
        key = (int(bool(lat.gh[1] and lat.gh[2])), max(send, recv))
        if key > best:
            best, best_r = key, r
    return best_r


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--config", default="q3", choices=sorted(bench.CONFIGS))
    ap.add_argument("--rank", type=int, default=None)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--profile-steps", type=int, default=10)
    ap.add_argument("--no-single", action="store_true", help="skip the 1-rank comparison")
    ap.add_argument("--kernel", default="auto", help="operator family (dofmap: the reference's "
                    "data model, with --geometry stored)")
    ap.add_argument("--geometry", default="auto")
    a = ap.parse_args(argv)
    degree, dpg, _, _ = bench.CONFIGS[a.config]
    nx = compute_mesh_size(dpg * a.ranks, degree)
    rank = pick_rank(a.ranks, nx, degree) if a.rank is None else a.rank
    lat = make_local_lattice(rank, a.ranks, nx, degree, whole_x=True)
    block = tuple(int(h - l) for l, h in zip(lat.c0, lat.c1))

    import torch

    from benchmark_dolfinx_amd.parallel.comm import Comm, EmulatedRankComm
    torch.cuda.set_device(0)
    ba = bench.parse_args(["--config", a.config])
    link = {k: float(os.environ.get(k, d)) for k, d in (("BDX_EMU_LINK_GBPS", 50.0),
                                                        ("BDX_EMU_LINK_LAT_US", 10.0),
                                                        ("BDX_EMU_ALLREDUCE_US", 20.0))}
    esz = 8 if bench.CONFIGS[a.config][2] == 64 else 4
    peers = {}
    for b in lat.halo_send_boxes() + lat.halo_recv_boxes():
        peers.setdefault(b.peer, [0, 0])
    for b in lat.halo_send_boxes():
        peers[b.peer][0] += b.size
    for b in lat.halo_recv_boxes():
        peers[b.peer][1] += b.size
    worst = max((max(s, r) for s, r in peers.values()), default=0) * esz
    model_us = worst / (link["BDX_EMU_LINK_GBPS"] * 1e3) + link["BDX_EMU_LINK_LAT_US"]

    def log(msg):
        print(f"[emulate] {msg}", file=sys.stderr, flush=True)

    comm = EmulatedRankComm(rank, a.ranks)
    rec = bench._measure(comm, ba, a.config, a.steps, a.warmup, profile_steps=a.profile_steps,
                         kernel=a.kernel, geometry=a.geometry, log=log)
    ph = rec.get("phases_ms") or {}
    out = {"mode": "emulated", "config": a.config, "nranks": a.ranks, "rank": rank,
           "mesh_global": list(nx), "block_cells": list(block), "ghost_planes": list(lat.gh),
           "link": link, "halo_peers": {str(k): v for k, v in sorted(peers.items())},
           "modelled_exchange_us": round(model_us, 1),
           "ms_per_step": rec["ms_per_step"], "ms_per_step_median": rec["ms_per_step_median"],
           "runtime": rec["runtime"], "kernel": rec["kernel"], "x_segments": rec["x_segments"],
           "phases_ms": ph,
           "comm_chain_done_ms": ph.get("t_halo_rev_done"),
           "interior_done_ms": ph.get("t_op_interior_done"),
           "margin_ms": (ph["t_op_interior_done"] - ph["t_halo_rev_done"]) if ph else None}
    print(json.dumps(out), flush=True)
    if not a.no_single:
        ba1 = bench.parse_args(["--config", a.config, "--mesh", ",".join(map(str, block))])
        r1 = bench._measure(Comm(), ba1, a.config, a.steps, a.warmup,
                            profile_steps=a.profile_steps, kernel=a.kernel,
                            geometry=a.geometry, log=log)
        print(json.dumps({"mode": "single", "config": a.config, "block_cells": list(block),
                          "ms_per_step": r1["ms_per_step"],
                          "ms_per_step_median": r1["ms_per_step_median"],
                          "kernel": r1["kernel"], "x_segments": r1["x_segments"],
                          "phases_ms": r1.get("phases_ms")}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
