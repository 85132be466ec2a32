#!/usr/bin/env python3
"""Full-size multi-rank rehearsal on one GPU: the bench's CG at --ranks x
--per-rank DoFs (threaded ranks, RCCL device-tensor rules emulated, native
runtime with the thread transport) against --ref-ranks ranks (default 1) on the
same global mesh.  The y_norm after the same number of iterations must agree
to rounding: partition invariance at the per-rank size of the driver's N-GPU
runs (e.g. --ranks 8 --ref-ranks 4 is the 2x2x2 geometry of N = 8).

    python scripts/fullsize_multirank.py [--config q3] [--per-rank 300000000]
                                         [--ranks 2] [--ref-ranks 1]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="q3")
    ap.add_argument("--per-rank", type=int, default=300_000_000)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ref-ranks", type=int, default=1,
                    help="rank count of the reference run on the same global mesh")
    a = ap.parse_args()
    import torch

    import bench
    from benchmark_dolfinx_amd.parallel.comm import run_threaded

    def job(comm, dpg):
        args = bench.parse_args(["--config", a.config, "--dofs-per-gpu", str(dpg), "--steps",
                                 str(a.steps), "--warmup", "2", "--gpus", str(comm.size),
                                 "--companions", "off", "--extras", "off"])
        out = bench.run(comm, args)
        torch.cuda.synchronize()
        return out

    total = a.per_rank * a.ranks
    res = {}
    for n in (a.ranks, a.ref_ranks):
        t0 = time.perf_counter()
        out = run_threaded(n, job, total // n, emulate="nccl")[0]
        torch.cuda.empty_cache()
        res[n] = out
        print(json.dumps({"ranks": n, "mesh": out["config"]["mesh"],
                          "ndofs": out["config"]["global_batch"],
                          "partition": out["config"]["parallelism"],
                          "runtime": out["config"]["runtime"],
                          "y_norm": out["config"]["y_norm"],
                          "phases_ms_max_over_ranks": out["config"]["phases_ms_max_over_ranks"],
                          "phases_per_rank": out["config"].get("phases_per_rank"),
                          "wall_s": round(time.perf_counter() - t0, 1)}), flush=True)
    y1, yn = res[a.ref_ranks]["config"]["y_norm"], res[a.ranks]["config"]["y_norm"]
    rel = abs(y1 - yn) / abs(y1)
    tol = 1e-11 if a.config != "q6f32" else 2e-5
    print(json.dumps({"rel_diff_y_norm": rel, "tol": tol, "ok": rel <= tol}), flush=True)
    return 0 if rel <= tol else 1


if __name__ == "__main__":
    raise SystemExit(main())
