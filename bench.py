#!/usr/bin/env python3
"""Headline benchmark: matrix-free CG on the Q_P Poisson problem, weak scaled.

BASELINE.json metric: "GDOF/s matrix-free Laplacian apply, Q3@300M & Q6@500M
dofs/GPU".  The reference's headline run is CG x 1000 iterations, FP64,
qmode=1 GLL, Q3 at 300 M DoFs per GPU (examples/Q3-300M.json: 257.544 GDoF/s
on 64 GH200 = 4.024 GDoF/s/GPU) and Q6 at 500 M DoFs per GPU (4.396).

One "step" = one CG iteration (one operator apply + 2 reductions + vector
updates), exactly the reference's rep (src/cg.hpp:121-167).
value = ndofs_global * K / (1e9 * t), t = MAX over ranks of the K-step time
(barrier + device sync on both sides).  Weak scaling: --dofs-per-gpu fixed.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config q3|q6|q6f32]
  torchrun --nproc-per-node N bench.py --gpus N ...

Data: synthetic by construction (the benchmark's own f and box mesh; no
checkpoint / dataset exists for this workload).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

CONFIGS = {
    # name: (degree, dofs_per_gpu, float bits, baseline GDoF/s per GPU or None)
    "q3": (3, 300_000_000, 64, 4.024),
    "q6": (6, 500_000_000, 64, 4.396),
    "q6f32": (6, 500_000_000, 32, None),
}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="q3", choices=sorted(CONFIGS))
    ap.add_argument("--dofs-per-gpu", type=int, default=None)
    ap.add_argument("--kernel", default="auto")
    ap.add_argument("--geometry", default="auto")
    ap.add_argument("--platform", default="gpu")
    ap.add_argument("--kappa", default="constant", choices=["constant", "random"],
                    help="per-cell random coefficients instead of the constant 2.0")
    return ap.parse_args(argv)


def run(comm, a) -> dict | None:
    """The timed CG benchmark on an initialised communicator; returns rank 0's
    JSON record (None elsewhere).  Callable in-process (tests run it on
    threaded ranks with RCCL semantics emulated)."""
    import torch

    from benchmark_dolfinx_amd.driver import make_operator
    from benchmark_dolfinx_amd.fem.mesh import compute_mesh_size
    from benchmark_dolfinx_amd.models.poisson import PoissonProblem
    from benchmark_dolfinx_amd.solvers.cg import DeviceCG, cg_solve

    degree, dpg, bits, base = CONFIGS[a.config]
    if a.dofs_per_gpu:
        dpg = a.dofs_per_gpu
    n = comm.size
    if n != a.gpus and comm.rank == 0:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {n}", file=sys.stderr)
    dtype = torch.float64 if bits == 64 else torch.float32
    nx = compute_mesh_size(dpg * n, degree)

    def log(msg):
        if comm.rank == 0:
            print(f"[bench {time.perf_counter() - t_setup:8.2f}s] {msg}", file=sys.stderr,
                  flush=True)

    t_setup = time.perf_counter()
    log(f"mesh {nx} degree {degree} fp{bits} on {n} rank(s)")
    pb = PoissonProblem(comm, nx, degree, 1, False, dtype, a.platform, 0.0, a.kappa)
    log("problem built")
    u = pb.assemble_rhs()
    x = pb.new_vector()
    log("rhs assembled")
    op = make_operator(pb, a.kernel, a.geometry)
    log(f"operator {getattr(op, 'name', type(op).__name__)} ready")
    gpu = a.platform == "gpu"

    def sync():
        if gpu:
            torch.cuda.synchronize()
        comm.barrier()
        if gpu:
            torch.cuda.synchronize()

    if gpu:
        cg = DeviceCG(pb)
        cg.start(op, x, u)
        cg.iterate(a.warmup)
    else:
        cg_solve(op, pb, x, u, a.warmup, 0.0)
    sync()
    log("warmup done")
    t_setup = time.perf_counter() - t_setup
    t0 = time.perf_counter()
    if gpu:
        cg.iterate(a.steps)
    else:
        cg_solve(op, pb, x, u, a.steps, 0.0)
    sync()
    dt = time.perf_counter() - t0
    dt = comm.allreduce_scalar(dt, "max")
    value = pb.ndofs_global * a.steps / (1e9 * dt)
    ynorm = pb.norm(x)
    runtime = (f"native C++ ({op._rt.transport}, hipGraph={op._rt.graphs})"
               if getattr(op, "_rt", None) is not None else "python")
    if hasattr(op, "close"):
        op.close()
    if comm.rank != 0:
        return None
    px, py, pz = pb.lat.pgrid
    return {
        "metric": "GDOF/s matrix-free Laplacian apply, Q3@300M & Q6@500M dofs/GPU, "
                  "1/2/4/8 MI355X",
        "value": value,
        "unit": "GDoF/s",
        "n_gpus": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * dt / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (value / (base * n)) if base else None,
        "dtype": "fp64" if bits == 64 else "fp32",
        "data": "synthetic (box mesh + f = 1000 exp(-((x-.5)^2+(y-.5)^2)/.02), "
                "as the reference)",
        "config": {
            "model": f"Q{degree} Poisson, qmode=1 GLL, matrix-free CG",
            "global_batch": pb.ndofs_global,
            "seq_len": degree,
            "parallelism": f"dd{n} ({px}x{py}x{pz} box partition)",
            "dofs_per_gpu": dpg,
            "mesh": list(nx),
            "kernel": getattr(op, "name", type(op).__name__),
            "geometry": getattr(op, "geometry", "otf"),
            "kappa": a.kappa,
            "runtime": runtime,
            "per_gpu_gdofs": value / n,
            "y_norm": ynorm,
            "setup_s": t_setup,
            "hiplib": os.path.basename(os.environ.get("BDX_HIP_LIB", "") or "libbdx_hip.so"),
        },
    }


def main(argv=None) -> int:
    a = parse_args(argv)
    from benchmark_dolfinx_amd.parallel.comm import finalize, init_distributed

    comm = init_distributed(a.platform)
    line = run(comm, a)
    if line is not None:
        print(json.dumps(line), flush=True)
    finalize()
    return 0


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    raise SystemExit(main())
