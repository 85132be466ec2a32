#!/usr/bin/env python3
"""Full-size multi-rank rehearsal on one GPU: the bench's CG at 2 x 300 M Q3
DoFs (2 threaded ranks, RCCL device-tensor rules emulated, native runtime with
the thread transport) against 1 rank on the same 600 M-DoF global mesh.  The
y_norm after the same number of iterations must agree to rounding (partition
invariance at the size the driver's N = 2 run uses).

    python scripts/fullsize_multirank.py [--config q3] [--per-rank 300000000]
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
    a = ap.parse_args()
    import torch

    import bench
    from benchmark_dolfinx_amd.parallel.comm import run_threaded

    def job(comm, dpg):
        args = bench.parse_args(["--config", a.config, "--dofs-per-gpu", str(dpg), "--steps",
                                 str(a.steps), "--warmup", "2", "--gpus", str(comm.size)])
        out = bench.run(comm, args)
        torch.cuda.synchronize()
        return out

    total = a.per_rank * a.ranks
    res = {}
    for n in (a.ranks, 1):
        t0 = time.perf_counter()
        out = run_threaded(n, job, total // n, emulate="nccl")[0]
        torch.cuda.empty_cache()
        res[n] = out
        print(json.dumps({"ranks": n, "mesh": out["config"]["mesh"],
                          "ndofs": out["config"]["global_batch"],
                          "partition": out["config"]["parallelism"],
                          "runtime": out["config"]["runtime"],
                          "y_norm": out["config"]["y_norm"],
                          "wall_s": round(time.perf_counter() - t0, 1)}), flush=True)
    y1, yn = res[1]["config"]["y_norm"], res[a.ranks]["config"]["y_norm"]
    rel = abs(y1 - yn) / abs(y1)
    tol = 1e-11 if a.config != "q6f32" else 2e-5
    print(json.dumps({"rel_diff_y_norm": rel, "tol": tol, "ok": rel <= tol}), flush=True)
    return 0 if rel <= tol else 1


if __name__ == "__main__":
    raise SystemExit(main())
