"""Does the split schedule's comm chain get CUs under a full interior launch?

At N > 1 the native runtime (csrc/hip/runtime.hip, CGRuntime::step) forks
the comm stream off the compute stream: forward halo send/recv -> the last
tile row and column (the tiles that read ghost planes) -> reverse send/recv,
while the compute stream runs one launch over every interior tile.  The
reference overlaps the same way (src/laplacian.hpp:281-349: scatter_fwd_begin,
interior cells, scatter_fwd_end, boundary cells).  The overlap only holds if
RCCL's kernels and the boundary launches are dispatched while the interior
grid still occupies the chip.

RCCL refuses two ranks on one GPU, so this replays the chain of a rank with y
and z ghost planes (the 1 x 2 x 4 split of N = 8) on a 1-rank RCCL
communicator: grouped self send/recv of that rank's halo volume at N = 8 (the
largest exchange of any of the 8 ranks at the weak-scaled mesh), the boundary
tiles, a second send/recv -- on the runtime's comm stream (greatest device
priority) -- concurrently with the interior tile rectangle of the same
300 M / 500 M DoF operator on the compute stream.  The chain must complete
before the interior launch does.  BDX_PROBE_OUT=<file> appends the record.

The emulated-rank test runs the real runtime of one N = 8 rank (its own
block, scripts/emulate_rank.py) with modelled xGMI link times.
"""

import json
import os

import pytest
import torch

from benchmark_dolfinx_amd.driver import make_operator
from benchmark_dolfinx_amd.fem.mesh import compute_mesh_size, make_local_lattice
from benchmark_dolfinx_amd.models.poisson import PoissonProblem
from benchmark_dolfinx_amd.parallel.comm import Comm
from benchmark_dolfinx_amd.solvers.cg import DeviceCG


def halo_elems_at(nranks: int, degree: int, dofs_per_gpu: int) -> int:
    """Largest one-way halo (elements) of any rank of the weak-scaled N-rank
    run, on the GPU partition (x kept whole)."""
    nx = compute_mesh_size(dofs_per_gpu * nranks, degree)
    best = 0
    for r in range(nranks):
        lat = make_local_lattice(r, nranks, nx, degree, whole_x=True)
        send = sum(b.size for b in lat.halo_send_boxes())
        recv = sum(b.size for b in lat.halo_recv_boxes())
        best = max(best, send, recv)
    return best


def test_halo_volume_at_8_ranks_is_plane_sized():
    n = halo_elems_at(8, 3, 300_000_000)
    # 1 x 2 x 4 split of the (441, 446, 451) Q3 mesh: one y plane + one z
    # plane of a 1324 x 669 x 338 block, ~1.3 M DoFs (10.7 MB in FP64)
    assert 1_000_000 < n < 1_600_000, n


@pytest.mark.gpu
@pytest.mark.parametrize("degree,dofs", [(3, 300_000_000), (6, 500_000_000)])
def test_comm_chain_completes_under_interior_launch(degree, dofs):
    torch.cuda.set_device(0)
    nelem = halo_elems_at(8, degree, dofs)
    pb = PoissonProblem(Comm(), compute_mesh_size(dofs, degree), degree, 1, False,
                        torch.float64, "gpu")
    u = pb.assemble_rhs()
    x = pb.new_vector()
    op = make_operator(pb, "auto", "auto")
    cg = DeviceCG(pb)
    cg.start(op, x, u)
    rt = op._rt
    assert rt is not None, "native runtime not loaded"
    prio = rt.comm_priority()
    rec = rt.overlap_probe(nelem, reps=5)
    rec.update(config=f"Q{degree} {pb.ndofs_global} DoFs fp64", kernel=op.name,
               nty=op.nty, ntz=op.ntz, nseg=op.nseg, priority=prio)
    print(json.dumps(rec))
    out = os.environ.get("BDX_PROBE_OUT")
    if out:
        with open(out, "a") as f:
            f.write(json.dumps(rec) + "\n")
    op.close()
    del op, cg, x, u, pb
    torch.cuda.empty_cache()
    assert rec["exchange_ok"], "RCCL self send/recv moved the wrong data"
    assert prio["comm_stream"] == prio["greatest"]
    # timing relations are recorded (BDX_PROBE_OUT, profiles/), not asserted:
    # box noise must not decide a correctness suite (the emulated-rank test
    # below and scripts/emulate_rank.py carry the schedule evidence)
    assert rec["chain_done_ms"] > 0 and rec["interior_done_ms"] > 0, rec


@pytest.mark.gpu
@pytest.mark.parametrize("config", ["q3", "q6"])
def test_emulated_rank_split_schedule(config, tmp_path):
    """One rank of the N = 8 weak-scaled run alone on this GPU: its own block
    (ghost planes, tile split, halo counts), the native runtime's split
    schedule with modelled link times (LinkEmuTransport) instead of RCCL.
    Asserts the structure (split schedule on, emulated transport, the link
    model applied); records the timeline (comm chain vs interior)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "scripts", "emulate_rank.py"), "--ranks", "8",
           "--config", config, "--steps", "10", "--warmup", "2", "--profile-steps", "4",
           "--no-single"]
    pr = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=root)
    assert pr.returncode == 0, pr.stderr[-2000:]
    rec = json.loads([ln for ln in pr.stdout.splitlines() if ln.startswith("{")][-1])
    print(json.dumps(rec))
    out = os.environ.get("BDX_PROBE_OUT")
    if out:
        with open(out, "a") as f:
            f.write(json.dumps(rec) + "\n")
    assert rec["mode"] == "emulated" and rec["nranks"] == 8
    assert "emulated" in rec["runtime"] and "overlap=True" in rec["runtime"], rec["runtime"]
    assert rec["ghost_planes"][1] and rec["ghost_planes"][2]
    ph = rec["phases_ms"]
    # the forward exchange took at least the modelled link time
    assert ph["halo_fwd"] >= 0.9 * rec["modelled_exchange_us"] * 1e-3, (ph, rec)
    assert rec["comm_chain_done_ms"] > 0 and rec["interior_done_ms"] > 0
    # loose structural check of the split schedule: the comm chain
    # (exchange, boundary tiles, ghost fold, reverse send) ends before the
    # interior tiles, with 0.25 ms of slack for box noise; measured margins
    # 1.98 ms (Q3) / 4.32 ms (Q6) (profiles/r5_split_schedule.md).  A chain
    # serialised behind the interior would end a whole chain later.
    assert rec["comm_chain_done_ms"] <= rec["interior_done_ms"] + 0.25, rec
