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

`python bench.py --gpus N` (N > 1, no torchrun environment) launches the N
ranks itself: this parent process starts N children with RANK / LOCAL_RANK /
WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, *before anything touches the GPU*
(it never imports torch), relays rank 0's JSON line, and kills the siblings
and exits non-zero if any child fails.  One rank per GPU, bound from
LOCAL_RANK (the reference runs one MPI rank per GPU, examples/submit.sh:16-19,
README.md:94-104).  N = 1 runs in-process, so a 1-GPU SCALE point is the
BENCH run.

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
    ap.add_argument("--perturb", type=float, default=0.0,
                    help="--geom_perturb_fact of the reference: random x-perturbation of "
                         "the vertices (general trilinear cells)")
    ap.add_argument("--mesh", default=None,
                    help="experiments only: explicit global cell counts NX,NY,NZ instead of "
                         "the config's DoF target")
    ap.add_argument("--profile-steps", type=int, default=5,
                    help="extra eager iterations with hipEvent phase timers (0: none)")
    ap.add_argument("--extras", default="auto", choices=["auto", "on", "off"],
                    help="after the headline run, time the same config with per-cell random "
                         "coefficients and on the perturbed (general trilinear) mesh and report "
                         "random_kappa_gdofs / general_gdofs (GPU platform only)")
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
    gpu = a.platform == "gpu"
    flags = None
    if gpu:
        from benchmark_dolfinx_amd.ops.native import build_flags
        flags = build_flags()
        if not flags["valid"] and os.environ.get("BDX_ALLOW_DROP") != "1":
            raise SystemExit(f"bench.py: the HIP library was built with timing-only phase "
                             f"drops {flags['drops']} (wrong numerics); refusing to time it "
                             f"(BDX_ALLOW_DROP=1 runs it, marked invalid)")
    dtype = torch.float64 if bits == 64 else torch.float32
    nx = (tuple(int(v) for v in a.mesh.split(",")) if a.mesh
          else compute_mesh_size(dpg * n, degree))

    t_log0 = time.perf_counter()

    def log(msg):
        if comm.rank == 0:
            print(f"[bench {time.perf_counter() - t_log0:8.2f}s] {msg}", file=sys.stderr,
                  flush=True)

    t_setup = time.perf_counter()
    phase_t = {}

    def mark(name):
        phase_t[name] = time.perf_counter() - t_setup - sum(phase_t.values())

    log(f"mesh {nx} degree {degree} fp{bits} on {n} rank(s)")
    pb = PoissonProblem(comm, nx, degree, 1, False, dtype, a.platform, a.perturb, a.kappa)
    log(f"problem built (partition {pb.lat.pgrid}, {pb.partition})")
    mark("problem")
    u = pb.assemble_rhs()
    x = pb.new_vector()
    log("rhs assembled")
    mark("rhs")
    op = make_operator(pb, a.kernel, a.geometry)
    log(f"operator {getattr(op, 'name', type(op).__name__)} ready")
    mark("operator")

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
        cg.wait()
    else:
        cg_solve(op, pb, x, u, a.warmup, 0.0)
    sync()
    log("warmup done")
    mark("warmup")
    t_setup = time.perf_counter() - t_setup
    t0 = time.perf_counter()
    if gpu:
        cg.iterate(a.steps)
        cg.wait()  # bounded by the RCCL deadline: a hung peer raises
    else:
        cg_solve(op, pb, x, u, a.steps, 0.0)
    sync()
    dt = time.perf_counter() - t0
    rank_dt = comm.gather_objects(dt)
    dt = comm.allreduce_scalar(dt, "max")
    value = pb.ndofs_global * a.steps / (1e9 * dt)
    ynorm = pb.norm(x)
    rt = getattr(op, "_rt", None)
    runtime = (f"native C++ ({rt.transport}, hipGraph={rt.graphs}, overlap={rt.overlap}, "
               f"tiled={rt.tiled})"
               if rt is not None else "python")
    comm_info = {"torch_backend": comm.backend, "torch_world": comm.size,
                 "transport": rt.transport if rt is not None else "python",
                 "rccl_ranks": rt.comm_ranks() if rt is not None else None,
                 "halo_overlap": rt.overlap if rt is not None else False,
                 "halo_bytes_per_exchange": pb.halo.bytes_per_exchange,
                 "rank_ms_per_step_max": 1e3 * max(rank_dt) / a.steps,
                 "rank_ms_per_step_min": 1e3 * min(rank_dt) / a.steps}
    # phase attribution: a few extra eager iterations with hipEvent timers,
    # after the timed loop and the norm (outside the measurement)
    phases = phases_max = None
    if rt is not None and a.profile_steps > 0:
        phases = rt.profile(a.profile_steps)
        allp = comm.gather_objects(phases)
        phases_max = {k: (all(p[k] for p in allp) if isinstance(phases[k], bool)
                          else max(p[k] for p in allp)) for k in phases}
    if hasattr(op, "close"):
        op.close()
    px, py, pz = pb.lat.pgrid
    mesh_nx, ndofs_global = list(nx), pb.ndofs_global
    kname = getattr(op, "name", type(op).__name__)
    geom = getattr(op, "geometry", "otf")
    xseg = getattr(op, "nseg", None)
    del op, x, u, pb, rt
    if gpu:
        del cg
        torch.cuda.empty_cache()
    extras = {}
    if gpu and a.extras in ("on", "auto"):
        # the north-star variants of the same config (BASELINE.json: random
        # coefficients; the reference's --geom_perturb_fact general cells)
        # "general" takes the auto kernel (fused3's x-trilinear instance on
        # these meshes); "general_trilinear" forces the fully general
        # trilinear-geometry instance on the same mesh
        for key, kappa, pert, geo in (("random_kappa", "random", a.perturb, a.geometry),
                                      ("general", a.kappa, a.perturb or 0.1, a.geometry),
                                      ("general_trilinear", a.kappa, a.perturb or 0.1,
                                       "otf-general")):
            extras[key] = _variant(comm, a, nx, degree, dtype, kappa, pert, sync, log, geo)
    if comm.rank != 0:
        return None
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
            "global_batch": ndofs_global,
            "seq_len": degree,
            "parallelism": f"dd{n} ({px}x{py}x{pz} box partition)",
            "dofs_per_gpu": dpg,
            "mesh": mesh_nx,
            "kernel": kname,
            "geometry": geom,
            "x_segments": xseg,
            "kappa": a.kappa,
            "geom_perturb_fact": a.perturb,
            "runtime": runtime,
            "per_gpu_gdofs": value / n,
            "y_norm": ynorm,
            "setup_s": t_setup,
            "setup_phases_s": phase_t,
            "device": _device_name() if gpu else "cpu",
            "build_flags": flags,
            "comm": comm_info,
            "phases_ms": phases,
            "phases_ms_max_over_ranks": phases_max,
        },
        "random_kappa_gdofs": extras.get("random_kappa", {}).get("value"),
        "general_gdofs": extras.get("general", {}).get("value"),
        "general_trilinear_gdofs": extras.get("general_trilinear", {}).get("value"),
        "variants": extras,
    }


def _variant(comm, a, nx, degree, dtype, kappa, perturb, sync, log, geometry) -> dict:
    """Time one variant of the headline config (same mesh and degree) with
    its own operator and CG; min(steps, 50) timed iterations after 3 warmup."""
    import torch

    from benchmark_dolfinx_amd.driver import make_operator
    from benchmark_dolfinx_amd.models.poisson import PoissonProblem
    from benchmark_dolfinx_amd.solvers.cg import DeviceCG

    pb = PoissonProblem(comm, nx, degree, 1, False, dtype, a.platform, perturb, kappa)
    u = pb.assemble_rhs()
    x = pb.new_vector()
    op = make_operator(pb, a.kernel, geometry)
    steps = min(a.steps, 50)
    cg = DeviceCG(pb)
    cg.start(op, x, u)
    cg.iterate(3)
    cg.wait()
    sync()
    t0 = time.perf_counter()
    cg.iterate(steps)
    cg.wait()
    sync()
    dt = comm.allreduce_scalar(time.perf_counter() - t0, "max")
    rec = {"value": pb.ndofs_global * steps / (1e9 * dt), "ms_per_step": 1e3 * dt / steps,
           "steps": steps, "kappa": kappa, "geom_perturb_fact": perturb,
           "kernel": getattr(op, "name", type(op).__name__),
           "geometry": getattr(op, "geometry", "otf"), "y_norm": pb.norm(x)}
    log(f"variant kappa={kappa} perturb={perturb}: {rec['value']:.2f} GDoF/s "
        f"({rec['kernel']}, {rec['geometry']})")
    if hasattr(op, "close"):
        op.close()
    del op, cg, x, u, pb
    torch.cuda.empty_cache()
    return rec


def _device_name() -> str:
    import torch

    from benchmark_dolfinx_amd.ops.kernels import device_name
    return device_name(torch.cuda.current_device())


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n: int, argv: list[str], port: int | None = None,
                 poll_s: float = 0.2) -> int:
    """Parent of a self-launched N-rank run (no torchrun).

    Runs in a process that has not initialised the GPU (torch is never
    imported here) and never execs: the children are fresh interpreters
    started with Popen.  Rank 0's stdout is relayed line by line (its JSON
    record is the last line); the other ranks' stdout is discarded and every
    rank's stderr is inherited.  The first child to fail takes the others
    down (exact PIDs, SIGTERM then SIGKILL) and its exit code is returned.
    """
    import signal
    import subprocess
    import threading

    port = port or _free_port()
    script = os.path.abspath(__file__)
    procs: list[subprocess.Popen] = []
    base = dict(os.environ)
    base.update(WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(port), GROUP_RANK="0", ROLE_RANK="0")
    base["PYTHONPATH"] = os.path.dirname(script) + os.pathsep + base.get("PYTHONPATH", "")
    if "OMP_NUM_THREADS" not in base:
        base["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // n))

    def _deathsig():  # children die with the parent (Linux prctl PR_SET_PDEATHSIG)
        try:
            import ctypes
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGKILL)
        except Exception:
            pass

    def _kill_all():
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()

    def _on_signal(signum, _frame):
        _kill_all()
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, _on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    relay = None
    try:
        for r in range(n):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            out = subprocess.PIPE if r == 0 else subprocess.DEVNULL
            procs.append(subprocess.Popen([sys.executable, script, *argv], env=env, stdout=out,
                                          text=True, preexec_fn=_deathsig))

        def _relay(stream):
            for line in stream:
                sys.stdout.write(line)
                sys.stdout.flush()

        relay = threading.Thread(target=_relay, args=(procs[0].stdout,), daemon=True)
        relay.start()
        rc = 0
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                print(f"[bench] a rank exited with {rc}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                _kill_all()
                break
            if all(c == 0 for c in codes):
                break
            time.sleep(poll_s)
        relay.join(timeout=10)
        return rc if rc >= 0 else 128 - rc
    finally:
        for s_, h in old.items():
            signal.signal(s_, h)


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    a = parse_args(argv)
    if os.environ.get("BDX_BENCH_FAIL_RANK") not in (None, "") and \
            os.environ.get("BDX_BENCH_FAIL_RANK") == os.environ.get("RANK"):
        print("bench.py: injected failure (BDX_BENCH_FAIL_RANK)", file=sys.stderr)
        return 3  # test hook: the launcher must take the other ranks down
    world = os.environ.get("WORLD_SIZE")
    if world is None and a.gpus > 1:
        return launch_ranks(a.gpus, argv)
    if world is not None and int(world) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}; refusing to report a "
              f"mis-sized run", file=sys.stderr)
        return 2
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
