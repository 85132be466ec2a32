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
import gc
import json
import os
import sys
import time

METRIC = "GDOF/s matrix-free Laplacian apply, Q3@300M & Q6@500M dofs/GPU, 1/2/4/8 MI355X"

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
    ap.add_argument("--companions", default="auto", choices=["auto", "on", "off"],
                    help="after the Q3 headline, time the metric's second half (Q6 at 500 M "
                         "DoFs/GPU, FP64 and FP32) and the headline with per-cell random "
                         "coefficients, each with the same steps/warmup, and report q6_gdofs / "
                         "q6f32_gdofs / random_kappa_gdofs (auto: on for the q3 config)")
    ap.add_argument("--extras", default="auto", choices=["auto", "on", "off"],
                    help="after the headline, time variants of it: the perturbed "
                         "(general trilinear) mesh, the "
                         "reference's data model (dofmap + stored G, Q3 and Q6, on its VALU "
                         "and its MFMA kernel), Q6 perturbed and Q6 FP32 perturbed (FP32 "
                         "MFMA) (GPU only; auto: on for one rank)")
    ap.add_argument("--box-probe", default="on", choices=["on", "off"],
                    help="after every timed run, measure the box's HBM stream rate "
                         "(untimed context: config.box_stream)")
    return ap.parse_args(argv)


def _median(v):
    s = sorted(v)
    n = len(s)
    return None if n == 0 else (s[n // 2] if n % 2 else 0.5 * (s[n // 2 - 1] + s[n // 2]))


def _pair_means(v):
    """Means of consecutive step pairs (a single step if fewer than two)."""
    if len(v) < 2:
        return list(v)
    return [0.5 * (v[i] + v[i + 1]) for i in range(0, len(v) - 1, 2)]


def _measure(comm, a, config, steps, warmup, *, kappa="constant", perturb=0.0,
             kernel="auto", geometry="auto", profile_steps=0, log=None) -> dict:
    """Build one config, run `warmup` untimed and `steps` timed CG
    iterations (barrier + device sync on both sides, MAX over ranks) and
    return its record (identical on every rank)."""
    import torch

    from benchmark_dolfinx_amd.driver import make_operator
    from benchmark_dolfinx_amd.fem.mesh import compute_mesh_size
    from benchmark_dolfinx_amd.models.poisson import PoissonProblem
    from benchmark_dolfinx_amd.solvers.cg import DeviceCG, cg_solve

    fail = os.environ.get("BDX_BENCH_FAIL_MEASURE", "")  # test hook: "<config>[:<kappa>]"
    if fail and fail in (config, f"{config}:{kappa}"):
        raise RuntimeError(f"injected failure in the {config} measurement")
    degree, dpg, bits, base = CONFIGS[config]
    if a.dofs_per_gpu:
        dpg = a.dofs_per_gpu
    n = comm.size
    gpu = a.platform == "gpu"
    dtype = torch.float64 if bits == 64 else torch.float32
    nx = (tuple(int(v) for v in a.mesh.split(",")) if a.mesh
          else compute_mesh_size(dpg * n, degree))
    log = log or (lambda msg: None)

    t_setup = time.perf_counter()
    phase_t = {}

    def mark(name):
        phase_t[name] = time.perf_counter() - t_setup - sum(phase_t.values())

    log(f"{config}: mesh {nx} degree {degree} fp{bits} on {n} rank(s), kappa={kappa} "
        f"perturb={perturb} kernel={kernel} geometry={geometry}")
    pb = PoissonProblem(comm, nx, degree, 1, False, dtype, a.platform, perturb, kappa)
    mark("problem")
    u = pb.assemble_rhs()
    x = pb.new_vector()
    mark("rhs")
    op = make_operator(pb, kernel, geometry)
    mark("operator")
    # one operator action on the RHS before the CG (untimed): the
    # cross-family consistency check of _record compares these scalars
    check = _action_check(pb, op, u)

    def sync():
        if gpu:
            torch.cuda.synchronize()
        comm.barrier()
        if gpu:
            torch.cuda.synchronize()

    cg = None
    preflight = None
    if gpu:
        cg = DeviceCG(pb)
        cg.start(op, x, u)
        rt0 = getattr(op, "_rt", None)
        if rt0 is not None and n > 1 and rt0.transport in ("rccl", "thread"):
            # the first exchange and all-reduce of the runtime's own RCCL
            # communicator, bounded well below the run deadline: a peer that
            # never joins surfaces here as an error, not as a hung warmup
            preflight = rt0.preflight(float(os.environ.get("BDX_PREFLIGHT_TIMEOUT_S", "120")))
            log(f"{config}: pre-flight exchange + all-reduce {preflight['ms']:.1f} ms")
        cg.iterate(warmup)
        cg.wait()
    else:
        cg_solve(op, pb, x, u, warmup, 0.0)
    sync()
    mark("warmup")
    t_setup = time.perf_counter() - t_setup
    t0 = time.perf_counter()
    step_ms = []
    if gpu:
        step_ms = cg.iterate_timed(steps)
        cg.wait()  # bounded by the RCCL deadline: a hung peer raises
    else:
        cg_solve(op, pb, x, u, steps, 0.0)
    sync()
    dt = time.perf_counter() - t0
    rank_dt = comm.gather_objects(dt)
    dt = comm.allreduce_scalar(dt, "max")
    value = pb.ndofs_global * steps / (1e9 * dt)
    # per-step device times over windows of two consecutive steps: fused5's
    # paired x update alternates a cheaper and a dearer step (runtime.hip)
    win = _pair_means(step_ms)
    med = _median(win)
    med = comm.allreduce_scalar(med, "max") if med is not None else None
    smin = comm.allreduce_scalar(min(win), "max") if win else None
    trace = os.environ.get("BDX_STEP_TRACE")
    if trace and comm.rank == 0:
        with open(trace, "a") as f:
            f.write(json.dumps({"config": config, "kernel": kernel, "perturb": perturb,
                                "step_ms": step_ms}) + "\n")
    ynorm = pb.norm(x)
    rt = getattr(op, "_rt", None)
    rec = {
        "value": value,
        "ms_per_step": 1e3 * dt / steps,
        "ms_per_step_median": med,
        "ms_per_step_min": smin,
        "steps": steps,
        "warmup": warmup,
        "vs_baseline": (value / (base * n)) if base else None,
        "dtype": "fp64" if bits == 64 else "fp32",
        "degree": degree,
        "dofs_per_gpu": dpg,
        "ndofs_global": pb.ndofs_global,
        "mesh": list(nx),
        "partition": list(pb.lat.pgrid),
        "kernel": getattr(op, "name", type(op).__name__),
        "geometry": getattr(op, "geometry", "otf"),
        "dofmap_core": getattr(op, "core", None),
        "x_segments": getattr(op, "nseg", None),
        "kappa": kappa,
        "geom_perturb_fact": perturb,
        "y_norm": ynorm,
        "action_check": check,
        "setup_s": t_setup,
        "setup_phases_s": phase_t,
        "runtime": (f"native C++ ({rt.transport}, hipGraph={rt.graphs}, overlap={rt.overlap}, "
                    f"tiled={rt.tiled})" if rt is not None else "python"),
        "comm": {"torch_backend": comm.backend, "torch_world": comm.size,
                 "transport": rt.transport if rt is not None else "python",
                 "rccl_ranks": rt.comm_ranks() if rt is not None else None,
                 "graphs": rt.graphs if rt is not None else False,
                 "halo_overlap": rt.overlap if rt is not None else False,
                 "halo_bytes_per_exchange": pb.halo.bytes_per_exchange,
                 "comm_stream_priority": rt.comm_priority() if rt is not None else None,
                 "preflight_ms": preflight["ms"] if preflight else None,
                 "rank_ms_per_step_max": 1e3 * max(rank_dt) / steps,
                 "rank_ms_per_step_min": 1e3 * min(rank_dt) / steps},
    }
    # phase attribution: a few extra eager iterations with hipEvent timers,
    # after the timed loop and the norm (outside the measurement)
    if rt is not None and profile_steps > 0:
        phases = rt.profile(profile_steps)
        allp = comm.gather_objects(phases)
        rec["phases_ms"] = phases
        rec["phases_ms_max_over_ranks"] = {
            k: (None if phases[k] is None else all(p[k] for p in allp)
                if isinstance(phases[k], bool) else max(p[k] for p in allp)) for k in phases}
        if n > 1:
            # per-rank timeline of the split schedule: when the comm-stream
            # chain (forward exchange, boundary tiles, reverse send) ended vs
            # the interior tiles, ms from the iteration start
            rec["phases_per_rank"] = [
                {"comm_chain_done": round(p["t_halo_rev_done"], 4),
                 "boundary_done": round(p["t_boundary_done"], 4),
                 "interior_done": round(p["t_op_interior_done"], 4),
                 "iteration": round(p["iteration"], 4),
                 "hidden": p["halo_rev_hidden"]} for p in allp]
    log(f"{config}: {value:.2f} GDoF/s ({rec['ms_per_step']:.3f} ms/step, median "
        f"{med if med is None else round(med, 3)} ms; {rec['kernel']}, {rec['geometry']})")
    if hasattr(op, "close"):
        op.close()
    del op, x, u, pb, rt, cg
    # the operator / runtime / problem objects hold reference cycles: collect
    # them now, so the next measurement (or an isolated child) gets the HBM
    # back (without this a --kernel dofmap run held ~200 GB of stale G and
    # vectors when its Q6 children started)
    gc.collect()
    if gpu:
        torch.cuda.empty_cache()
    return rec


def _emulated_prediction(config: str, kernel: str, n: int):
    """ms per step that one rank of this N-rank run measured ALONE on one GPU
    with modelled 50 GB/s + 10 us links (scripts/emulate_rank.py, committed in
    benchmark_dolfinx_amd/data/emulated_predictions.json): context for the
    first real multi-GPU curve, never part of a timed value.  None if that
    (config, kernel, N) was not emulated."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "benchmark_dolfinx_amd",
                        "data", "emulated_predictions.json")
    try:
        with open(path) as f:
            tab = json.load(f)
        return tab["runs"][config][kernel][str(n)]
    except (OSError, KeyError, ValueError):
        return None


def _action_check(pb, op, u) -> dict:
    """z = A b once (the operator's action mode, before any CG state exists)
    and two scalars of it: ||z||_2 and sum_i w_i z_i^2 with w_i = 1 + sin(0.7 i
    + 0.3) / 2 over the storage index (owned dofs; positive weights, so the
    sum does not cancel and a misplaced entry changes it).  Families that implement the same
    operator on the same partition must agree to rounding (~1e-14); unlike the
    CG iterate's norm, which drifts with the summation order over hundreds of
    iterations (Q6 at 210 iterations: 5e-6 between two runs of the SAME
    kernel on different boxes, profiles/r5*_bench_default.json), this pins
    the operator itself."""
    import torch
    z = pb.new_vector()
    op.apply(u, z)
    if z.is_cuda:
        torch.cuda.synchronize()
    w = 1.0 + 0.5 * torch.sin(torch.arange(z.numel(), dtype=torch.float64, device=z.device) * 0.7
                              + 0.3)
    w = w.view(z.shape) * z.double()
    out = {"norm": pb.norm(z), "wdot": pb.inner(z, w)}
    del z, w
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    return out


# Pairs of records that time the same problem with different operator
# families (headline / companion key, variant key): their action checks must
# agree to CONSISTENCY_TOL, else the run fails.
CONSISTENCY_PAIRS = (("q3", "dofmap"), ("q6", "q6_dofmap"), ("general", "general_trilinear"),
                     ("dofmap", "dofmap_mfma"), ("q6_dofmap", "q6_dofmap_mfma"))
CONSISTENCY_TOL = 1e-9
YNORM_TOL = 1e-4  # CG iterates: rounding drift over hundreds of iterations (see above)


def _consistency(head, companions, extras) -> dict:
    """Relative gaps of the action checks and of the CG iterate norms for the
    CONSISTENCY_PAIRS present in this run; `ok` is False if any gap exceeds
    its tolerance (action: 1e-9 in FP64, 1e-5 in FP32; y_norm: 1e-4)."""
    recs = {"q3": head if head.get("degree") == 3 else None, **companions, **extras}
    if head.get("degree") == 6:
        recs.setdefault("q6", head)
    out = {"tol_action": CONSISTENCY_TOL, "tol_y_norm": YNORM_TOL, "pairs": {}, "ok": True}
    for a_key, b_key in CONSISTENCY_PAIRS:
        ra, rb = recs.get(a_key), recs.get(b_key)
        if not ra or not rb or ra.get("value") is None or rb.get("value") is None:
            continue
        ca, cb = ra.get("action_check"), rb.get("action_check")
        if ra.get("geom_perturb_fact") != rb.get("geom_perturb_fact") or \
                ra.get("kappa") != rb.get("kappa"):
            continue
        gaps = {}
        if ca and cb:
            for k in ("norm", "wdot"):
                gaps[f"action_{k}"] = abs(ca[k] - cb[k]) / max(abs(cb[k]), 1e-300)
        if ra.get("y_norm") is not None and rb.get("y_norm") is not None and \
                ra.get("steps") == rb.get("steps") and ra.get("warmup") == rb.get("warmup"):
            gaps["y_norm"] = abs(ra["y_norm"] - rb["y_norm"]) / max(abs(rb["y_norm"]), 1e-300)
        tol = CONSISTENCY_TOL if ra.get("dtype", "fp64") == "fp64" else 1e-5
        ok = all(v <= (YNORM_TOL if k == "y_norm" else tol) for k, v in gaps.items())
        out["pairs"][f"{a_key}~{b_key}"] = {
            "kernels": [ra.get("kernel"), rb.get("kernel")],
            **{k: float(f"{v:.3e}") for k, v in gaps.items()}, "ok": ok}
        out["ok"] = out["ok"] and ok
    return out


def _measure_env(comm, a, config, steps, warmup, *, extra_env=None, **kw) -> dict:
    """`_measure` in this process with `extra_env` set for its duration."""
    old = {k: os.environ.get(k) for k in (extra_env or {})}
    os.environ.update(extra_env or {})
    try:
        return _measure(comm, a, config, steps, warmup, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _measure_isolated(a, config, steps, warmup, *, kappa="constant", perturb=0.0,
                      kernel="auto", geometry="auto", extra_env=None, log=None) -> dict:
    """One-rank `_measure` in a child interpreter (this script, headline only,
    no companions / variants; `extra_env`: added to the child's environment); returns
    the child's record with its own clock.  The parent has released its
    cached device memory, and never execs: the child is a fresh process
    started with Popen semantics."""
    import subprocess

    argv = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--config", config,
            "--steps", str(steps), "--warmup", str(warmup), "--companions", "off",
            "--extras", "off", "--box-probe", "off", "--profile-steps", "0", "--kappa", kappa,
            "--perturb", repr(float(perturb)), "--kernel", kernel, "--geometry", geometry,
            "--platform", a.platform]
    if a.dofs_per_gpu:
        argv += ["--dofs-per-gpu", str(a.dofs_per_gpu)]
    if a.mesh:
        argv += ["--mesh", a.mesh]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "ROLE_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env or {})
    timeout = float(os.environ.get("BDX_BENCH_CHILD_TIMEOUT_S", "600"))
    pr = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=timeout)
    for line in pr.stderr.splitlines():
        if log and line.startswith("[bench"):
            log("  (child) " + line.split("] ", 1)[-1])
    lines = [ln for ln in pr.stdout.splitlines() if ln.startswith("{")]
    if pr.returncode != 0 or not lines:
        raise RuntimeError(f"isolated {config} measurement exited {pr.returncode}: "
                           f"{pr.stderr.strip()[-400:]}")
    d = json.loads(lines[-1])
    if d.get("value") is None:
        raise RuntimeError(f"isolated {config} measurement failed: {d.get('error')}")
    c = d["config"]
    return {"value": d["value"], "ms_per_step": d["ms_per_step"],
            "ms_per_step_median": d["ms_per_step_median"],
            "ms_per_step_min": d["ms_per_step_min"], "steps": d["steps"], "warmup": d["warmup"],
            "vs_baseline": d["vs_baseline"], "dtype": d["dtype"], "dofs_per_gpu": c["dofs_per_gpu"],
            "ndofs_global": c["global_batch"], "mesh": c["mesh"], "kernel": c["kernel"],
            "geometry": c["geometry"], "dofmap_core": c.get("dofmap_core"),
            "x_segments": c["x_segments"], "kappa": c["kappa"],
            "geom_perturb_fact": c["geom_perturb_fact"], "y_norm": c["y_norm"],
            "action_check": c.get("action_check"),
            "setup_s": c["setup_s"], "runtime": c["runtime"], "isolated_process": True}


class MeasurementFailed(RuntimeError):
    """A measurement failed on a multi-rank run: fatal (the other ranks may
    be inside a collective the failed rank will never join), but it carries
    the records measured so far (headline, companions, variants) so rank 0
    can still report them."""

    def __init__(self, msg, partial):
        super().__init__(msg)
        self.partial = partial


def _guarded(comm, fn, log) -> dict:
    """Run one secondary measurement.  On one rank an error is recorded, not
    raised, so the already measured headline is always reported.  With
    several ranks it is re-raised: a rank that skipped ahead would start the
    next measurement while its peers are still inside the failed one's
    collectives (they would block until the deadline or pair up the wrong
    collectives)."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 - reported in the JSON
        if comm.size > 1:
            raise
        log(f"secondary measurement failed: {e!r}")
        try:
            import torch
            gc.collect()  # what the failed measurement left in reference cycles
            if torch.cuda.is_available():
                torch.cuda.empty_cache()
        except Exception:  # noqa: BLE001
            pass
        return {"value": None, "error": repr(e)}


def run(comm, a) -> dict | None:
    """The timed CG benchmark on an initialised communicator; returns rank 0's
    JSON record (None elsewhere).  Callable in-process (tests run it on
    threaded ranks with RCCL semantics emulated)."""
    n = comm.size
    gpu = a.platform == "gpu"
    flags = None
    if gpu:
        from benchmark_dolfinx_amd.ops.native import build_flags
        flags = build_flags()
        if not flags["valid"] and os.environ.get("BDX_ALLOW_VARIANT") != "1":
            raise SystemExit(f"bench.py: the loaded HIP library is not the production build "
                             f"({flags}); refusing to time it (BDX_ALLOW_VARIANT=1 runs it, "
                             f"marked invalid)")
    t_log0 = time.perf_counter()

    def log(msg):
        if comm.rank == 0:
            print(f"[bench {time.perf_counter() - t_log0:8.2f}s] {msg}", file=sys.stderr,
                  flush=True)

    head = _measure(comm, a, a.config, a.steps, a.warmup, kappa=a.kappa, perturb=a.perturb,
                    kernel=a.kernel, geometry=a.geometry, profile_steps=a.profile_steps,
                    log=log)
    # the metric's second half (Q6 at 500 M DoFs/GPU, FP64 and FP32) and the
    # north star's random coefficients on the headline config, each on the
    # headline's clock discipline (own steps / warmup / ms_per_step), at
    # every rank count
    companions = {}
    if a.companions == "on" or (a.companions == "auto" and a.config == "q3" and not a.mesh):
        # random kappa first, on the headline's problem size: after the 500 M
        # DoF Q6 problems its vectors land on fragmented device memory and it
        # measured 7 % slower than the same run in a fresh process (55.5 vs
        # 58.5-59.3 GDoF/s, round 4), a placement artefact, not the kernel
        specs = [("random_kappa", a.config, "random")] if a.kappa == "constant" else []
        specs += [(c, c, a.kappa) for c in ("q6", "q6f32")]
        for key, c, kap in specs:
            try:
                companions[key] = _guarded(comm, lambda c=c, kap=kap: _measure(
                    comm, a, c, a.steps, a.warmup, kappa=kap, perturb=a.perturb,
                    kernel=a.kernel, geometry=a.geometry, log=log), log)
            except Exception as e:
                raise MeasurementFailed(f"{key}: {e!r}", (head, companions, {})) from e
    extras = {}
    if a.extras == "auto" and n > 1 and a.config == "q3" and not a.mesh:
        # N > 1: the reference's own data model (dofmap + stored G, the
        # layout of its published 64-rank runs, /root/reference/src/
        # laplacian.hpp:281-349) on this weak-scaled mesh, in-process after
        # the companions, at the headline's steps / warm-up, with its per-rank
        # split-schedule timeline; on the CPU platform
        # the same record comes from the C++ dofmap operator (DofmapLaplacianCPU)
        try:
            extras["dofmap"] = _guarded(comm, lambda: _measure(
                comm, a, a.config, a.steps, a.warmup, kappa=a.kappa, perturb=a.perturb,
                kernel="dofmap", geometry="stored", profile_steps=a.profile_steps, log=log), log)
        except Exception as e:
            raise MeasurementFailed(f"dofmap: {e!r}", (head, companions, extras)) from e
        if extras["dofmap"].get("value") is not None:
            extras["dofmap"]["emulated_ms_per_step"] = _emulated_prediction(a.config, "dofmap", n)
    elif gpu and (a.extras == "on" or (a.extras == "auto" and n == 1)):
        # north-star variants of the headline config (BASELINE.json: random
        # coefficients; the reference's --geom_perturb_fact general cells; the
        # reference's own data model).  "general" takes the auto kernel
        # (fused3's x-trilinear instance on these meshes); "general_trilinear"
        # forces the fully general trilinear-geometry instance on the same
        # mesh; "dofmap" runs explicit cell->dof / cell->vertex arrays with G
        # stored per quadrature point, as the reference does.
        # the headline's clock discipline: same --steps / --warmup
        pert = a.perturb or 0.1
        specs = (("general", a.config, dict(kappa=a.kappa, perturb=pert)),
                 ("general_trilinear", a.config, dict(kappa=a.kappa, perturb=pert,
                                                      geometry="otf-general")),
                 ("dofmap", a.config, dict(kappa=a.kappa, perturb=a.perturb, kernel="dofmap",
                                           geometry="stored")),
                 ("q6_general", "q6", dict(kappa=a.kappa, perturb=pert)),
                 ("q6_dofmap", "q6", dict(kappa=a.kappa, perturb=a.perturb, kernel="dofmap",
                                          geometry="stored")),
                 # BASELINE configs[4] "MFMA f32 tensor contractions": fused3's
                 # FP32 x-trilinear instance, whose y / z stages run on
                 # v_mfma_f32_16x16x4_f32 (lap_fused3.h kF3MfmaF32)
                 ("q6f32_general", "q6f32", dict(kappa=a.kappa, perturb=pert)),
                 # the reference data model with every contraction on
                 # v_mfma_f64_16x16x4_f64 (lap_dofmfma.h; selectable, not the
                 # default: profiles/r6_dofmap_mfma.md), same problems as
                 # "dofmap" / "q6_dofmap", checked against them below
                 ("dofmap_mfma", a.config, dict(kappa=a.kappa, perturb=a.perturb,
                                                kernel="dofmap", geometry="stored",
                                                extra_env={"BDX_DOFMAP_MFMA": "1"})),
                 ("q6_dofmap_mfma", "q6", dict(kappa=a.kappa, perturb=a.perturb, kernel="dofmap",
                                               geometry="stored",
                                               extra_env={"BDX_DOFMAP_MFMA": "1"})))
        # Each variant runs in a fresh child process on one rank: in this
        # process, after the headline and the 500 M DoF companions, the
        # variants measured up to 15 % low (dofmap Q3 11.9 vs 14.0 GDoF/s on
        # one box, round 4) -- device memory handed out after many large
        # allocations and frees, not the kernels.  BDX_BENCH_ISOLATE=0 keeps
        # them in-process.
        isolate = n == 1 and os.environ.get("BDX_BENCH_ISOLATE", "1") != "0"
        for key, cfg, kw in specs:
            if cfg != a.config and (a.mesh or a.config != "q3"):
                continue
            kw.setdefault("kernel", a.kernel if kw.get("geometry") is None else "auto")
            kw.setdefault("geometry", a.geometry)
            try:
                if isolate:
                    extras[key] = _guarded(comm, lambda cfg=cfg, kw=kw: _measure_isolated(
                        a, cfg, a.steps, a.warmup, log=log, **kw), log)
                else:
                    extras[key] = _guarded(comm, lambda cfg=cfg, kw=kw: _measure_env(
                        comm, a, cfg, a.steps, a.warmup, log=log, **kw), log)
            except Exception as e:
                raise MeasurementFailed(f"{key}: {e!r}", (head, companions, extras)) from e
    if gpu and a.box_probe == "on":
        try:
            head["box_stream"] = _guarded(comm, lambda: _stream_probe(comm, head["dofs_per_gpu"]),
                                          log)
        except Exception as e:
            raise MeasurementFailed(f"box_stream: {e!r}", (head, companions, extras)) from e
    if comm.rank != 0:
        return None
    return _record(a, n, head, companions, extras, flags, gpu)


def _stream_probe(comm, n: int, reps: int = 10) -> dict:
    """The box's HBM stream rate, measured after every timed run (context, not
    part of any timed region): r += a y over the headline's n doubles per GPU,
    2 reads + 1 write, the CG update pass's access pattern.  Boxes of this pool
    differ by 7-12 % on the stream-bound configs (Q3, the dofmap data model)
    while the compute-side Q6 ones do not (profiles/r5_final_repeat.md); this
    puts the box's rate next to the number.  TB/s, min / max over ranks; and
    the box's DGEMM rate (TFLOP/s) as its compute-side counterpart."""
    import torch
    r = torch.ones(n, dtype=torch.float64, device="cuda")
    y = torch.ones_like(r)
    r.add_(y, alpha=-1e-9)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        r.add_(y, alpha=-1e-9)
    e1.record()
    torch.cuda.synchronize()
    tbps = 24.0 * n * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12
    del r, y
    # the box's FP64 compute rate next to it: a 4096^3 DGEMM (rocBLAS), the
    # side that the compute-heavy configs (Q6, perturbed) lean on
    m = 4096
    a_ = torch.rand(m, m, dtype=torch.float64, device="cuda")
    b_ = torch.rand(m, m, dtype=torch.float64, device="cuda")
    c_ = a_ @ b_
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        torch.mm(a_, b_, out=c_)
    e1.record()
    torch.cuda.synchronize()
    tflops = 2.0 * m ** 3 * reps / (e0.elapsed_time(e1) * 1e-3) / 1e12
    del a_, b_, c_
    torch.cuda.empty_cache()
    return {"op": "r += a*y, fp64, 2R1W", "n": n,
            "tbps_min": -comm.allreduce_scalar(-tbps, "max"),
            "tbps_max": comm.allreduce_scalar(tbps, "max"),
            "dgemm_tflops_min": -comm.allreduce_scalar(-tflops, "max"),
            "dgemm_tflops_max": comm.allreduce_scalar(tflops, "max")}


def _record(a, n, head, companions, extras, flags, gpu) -> dict:
    """Rank 0's JSON line."""
    degree = head["degree"]
    px, py, pz = head["partition"]
    return {
        "metric": METRIC,
        "value": head["value"],
        "unit": "GDoF/s",
        "n_gpus": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": head["ms_per_step"],
        "ms_per_step_median": head["ms_per_step_median"],
        "ms_per_step_min": head["ms_per_step_min"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": head["vs_baseline"],
        "dtype": head["dtype"],
        "data": "synthetic (box mesh + f = 1000 exp(-((x-.5)^2+(y-.5)^2)/.02), "
                "as the reference)",
        "config": {
            "model": f"Q{degree} Poisson, qmode=1 GLL, matrix-free CG",
            "global_batch": head["ndofs_global"],
            "seq_len": degree,
            "parallelism": f"dd{n} ({px}x{py}x{pz} box partition)",
            "dofs_per_gpu": head["dofs_per_gpu"],
            "mesh": head["mesh"],
            "kernel": head["kernel"],
            "geometry": head["geometry"],
            "dofmap_core": head.get("dofmap_core"),
            "x_segments": head["x_segments"],
            "kappa": head["kappa"],
            "geom_perturb_fact": head["geom_perturb_fact"],
            "runtime": head["runtime"],
            "per_gpu_gdofs": head["value"] / n,
            "y_norm": head["y_norm"],
            "action_check": head.get("action_check"),
            "setup_s": head["setup_s"],
            "setup_phases_s": head["setup_phases_s"],
            "device": _device_name() if gpu else "cpu",
            "build_flags": flags,
            "comm": head["comm"],
            "phases_ms": head.get("phases_ms"),
            "phases_ms_max_over_ranks": head.get("phases_ms_max_over_ranks"),
            "phases_per_rank": head.get("phases_per_rank"),
            "box_stream": head.get("box_stream"),
            "emulated_ms_per_step": (_emulated_prediction(a.config, head["kernel"], n)
                                     if n > 1 else None),
        },
        "q6_gdofs": companions.get("q6", {}).get("value"),
        "q6f32_gdofs": companions.get("q6f32", {}).get("value"),
        "companions": companions,
        "random_kappa_gdofs": companions.get("random_kappa", {}).get("value"),
        "general_gdofs": extras.get("general", {}).get("value"),
        "general_trilinear_gdofs": extras.get("general_trilinear", {}).get("value"),
        "dofmap_gdofs": extras.get("dofmap", {}).get("value"),
        "q6_general_gdofs": extras.get("q6_general", {}).get("value"),
        "q6_dofmap_gdofs": extras.get("q6_dofmap", {}).get("value"),
        "q6f32_general_gdofs": extras.get("q6f32_general", {}).get("value"),
        "dofmap_mfma_gdofs": extras.get("dofmap_mfma", {}).get("value"),
        "q6_dofmap_mfma_gdofs": extras.get("q6_dofmap_mfma", {}).get("value"),
        "variants": extras,
        "consistency": _consistency(head, companions, extras),
    }


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

        relayed = []

        def _relay(stream):
            for line in stream:
                if line.startswith("{"):
                    relayed.append(line)
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
        rc = rc if rc >= 0 else 128 - rc
        if rc and not relayed:
            # rank 0 never got to report (it was taken down with a failed
            # peer): the one JSON line says so instead of leaving stdout empty
            print(json.dumps({"metric": METRIC, "value": None, "unit": "GDoF/s", "n_gpus": n,
                              "higher_is_better": True, "scaling": "weak",
                              "error": f"a rank exited with {rc} before rank 0 reported"}),
                  flush=True)
        return rc
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
    try:
        line = run(comm, a)
    except Exception as e:
        # one JSON line with the error (and whatever was measured before it)
        # instead of a silent non-zero exit; the process still fails
        if comm.rank == 0:
            rec = {"metric": METRIC, "value": None, "unit": "GDoF/s", "n_gpus": a.gpus,
                   "steps": a.steps, "warmup": a.warmup, "higher_is_better": True,
                   "scaling": "weak", "error": repr(e)}
            part = getattr(e, "partial", None)
            if part is not None:
                try:
                    rec.update(_record(a, comm.size, part[0], part[1], part[2], None,
                                       a.platform == "gpu"))
                    rec["error"] = repr(e)
                except Exception:  # noqa: BLE001 - the error line must go out
                    pass
            print(json.dumps(rec), flush=True)
        print(f"bench.py: rank {comm.rank}: {e!r}", file=sys.stderr, flush=True)
        return 1
    rc = 0
    if line is not None:
        print(json.dumps(line), flush=True)
        cons = line.get("consistency") or {}
        if not cons.get("ok", True):
            bad = {k: v for k, v in cons["pairs"].items() if not v["ok"]}
            print(f"bench.py: operator families disagree on the same problem: {bad}",
                  file=sys.stderr, flush=True)
            rc = 4
    finalize()
    return rc


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    raise SystemExit(main())
