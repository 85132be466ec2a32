"""Benchmark drivers: setup -> timed loop -> norms -> optional CSR comparison.

Reference: `laplace_action_gpu` / `laplace_action_cpu`
(src/laplacian_solver.cpp:64-391) and `run_benchmark` (src/main.cpp:41-133).

Timing fixes quirk Q9: all ranks synchronise the device and meet at a
barrier before the clock starts and after it stops, and the reported time is
the MAX over ranks (the reference reads rank 0's clock with no barrier).
"""

from __future__ import annotations

import os
import time
from dataclasses import dataclass, field

import torch

from .models.poisson import (CSROperator, MatFreeLaplacianCPU, MatFreeLaplacianGPU,
                             PoissonProblem)
from .solvers.cg import DeviceCG, cg_solve
from .utils.timing import add_time, timed


@dataclass
class BenchmarkResults:
    mat_free_time: float = 0.0
    unorm: float = 0.0
    ynorm: float = 0.0
    znorm: float = 0.0
    enorm: float = 0.0
    extra: dict = field(default_factory=dict)


def make_operator(pb: PoissonProblem, kernel: str = "auto", geometry: str = "auto"):
    if pb.platform == "cpu":
        if kernel == "dofmap":
            # the reference's own CPU data model (cell -> dof map, stored G)
            from .models.unstructured import DofmapLaplacianCPU
            return DofmapLaplacianCPU(pb, "otf" if geometry == "otf" else "stored")
        return MatFreeLaplacianCPU(pb)
    if kernel == "auto":
        # measured on MI355X (profiles/): fused3 wins on parallelepiped meshes
        # (Q3 +4 %, Q6 +12 % over fused2); on general trilinear meshes its
        # larger register footprint spills at Q3, so fused2 takes those
        if geometry == "stored":
            kernel = "fused" if pb.kc is None else "v1"
        elif geometry == "otf-general" or not pb.all_affine:
            # general (trilinear) cells, same-box A/B (scripts/job_r2i.sh,
            # job_r2r.sh): Q3 fused3 18.2 vs fused2 16.5 GDoF/s; Q6 fused3
            # 22.0 (spill-free) vs fused2 18.8; fused3 falls back to fused2
            # where it does not apply (phi0 = I).  On the reference's
            # x-perturbed meshes both take their x-trilinear instance
            # (profiles/r2_xtrilinear.md: Q3 26.2, Q6 29.1 GDoF/s)
            kernel = "fused3"
        else:
            # fused5 (nodal Kronecker sum factorisation) on axis-aligned boxes
            # at every P >= 3 (the benchmark mesh); parallelepipeds with a full
            # Jacobian take fused3's affine instance.  The fused4 MFMA
            # Kronecker core (beaten by fused5 at Q3 FP64 since
            # profiles/r2_launder.md: 58.4 vs 52.1 GDoF/s) and fused5's
            # sheared-cell instance were reachable only from a test-only
            # shear map and were removed in round 5.
            from .models.fused import fused_supported
            auto = "fused5" if fused_supported(pb, 5) else "fused3"
            kernel = os.environ.get("BDX_AUTO_AFFINE", auto)
    if kernel == "dofmap":
        # the unstructured data model: explicit cell->dof / cell->vertex maps
        from .models.unstructured import DofmapLaplacianGPU
        return DofmapLaplacianGPU(pb, "stored" if geometry == "stored" else "otf")
    if kernel == "fused5":
        from .models.fused import FusedLaplacianGPU, fused_supported
        if fused_supported(pb, 5) and geometry in ("auto", "otf"):
            return FusedLaplacianGPU(pb, geometry="otf", version=5)
        kernel = "fused3"
    if kernel == "fused3":
        from .models.fused import FusedLaplacianGPU, fused_supported
        if fused_supported(pb, 3) and geometry in ("auto", "otf", "otf-general"):
            # "otf-general" forces the general trilinear instance; "auto" takes
            # the x-trilinear one on the reference's perturbed meshes
            return FusedLaplacianGPU(pb, geometry="otf", version=3,
                                     affine=geometry != "otf-general",
                                     xtri=geometry != "otf-general")
        kernel = "fused2"
    if kernel == "fused2":
        from .models.fused import FusedLaplacianGPU, fused_supported
        if fused_supported(pb, 2) and geometry in ("auto", "otf", "otf-general"):
            return FusedLaplacianGPU(pb, geometry="otf", version=2,
                                     affine=geometry != "otf-general",
                                     xtri=geometry != "otf-general")
        kernel = "fused"
    if geometry == "otf-general":
        geometry = "otf"
    if kernel == "fused":
        from .models.fused import FusedLaplacianGPU, fused_supported
        if fused_supported(pb) and pb.kc is None:
            return FusedLaplacianGPU(pb, geometry="otf" if geometry == "auto" else geometry)
        kernel = "v1"
    if kernel == "v1":
        return MatFreeLaplacianGPU(pb, geometry="stored" if geometry == "auto" else geometry)
    raise ValueError(f"unknown kernel {kernel}")


def _sync(pb: PoissonProblem) -> None:
    if pb.platform == "gpu":
        torch.cuda.synchronize()
    pb.comm.barrier()
    if pb.platform == "gpu":
        torch.cuda.synchronize()


def _run_loop(op, pb, x, u, nreps, use_cg, dev_cg):
    if use_cg:
        if pb.platform == "gpu":
            dev_cg.solve(op, x, u, nreps)
            dev_cg.wait()  # bounded by the RCCL deadline (native runtime)
        else:
            cg_solve(op, pb, x, u, nreps, 0.0)
    else:
        for _ in range(nreps):
            op.apply(u, x)


def laplace_action(pb: PoissonProblem, nreps: int, use_cg: bool, mat_comp: bool,
                   kernel: str = "auto", geometry: str = "auto", warmup: int = 0,
                   printer=print) -> BenchmarkResults:
    rank0 = pb.comm.rank == 0
    res = BenchmarkResults()
    u = pb.assemble_rhs()
    y = pb.new_vector()
    with timed("% Create matfree operator"):
        op = make_operator(pb, kernel, geometry)
        if pb.platform == "gpu":
            torch.cuda.synchronize()
    dev_cg = DeviceCG(pb) if (use_cg and pb.platform == "gpu") else None
    res.extra["kernel"] = getattr(op, "name", type(op).__name__)
    res.extra["geometry"] = getattr(op, "geometry", "otf")
    if warmup > 0:
        with timed("~warmup"):
            _run_loop(op, pb, y, u, warmup, use_cg, dev_cg)
            y.zero_()
    _sync(pb)
    t0 = time.perf_counter()
    _run_loop(op, pb, y, u, nreps, use_cg, dev_cg)
    _sync(pb)
    dt = time.perf_counter() - t0
    dt = pb.comm.allreduce_scalar(dt, "max")
    add_time("% Matrix-free " + ("CG" if use_cg else "action"), dt, 1)
    res.mat_free_time = dt
    res.unorm = pb.norm(u)
    res.ynorm = pb.norm(y)
    if rank0:
        comp = "CG" if use_cg else "Action"
        printer(f"Computation time ({comp}): {dt:.6g}s")
        printer(f"Computation rate (Gdofs/s): {pb.ndofs_global * nreps / (1e9 * dt):.6g}")
        printer(f"Norm of u = {res.unorm:.6g}")
        printer(f"Norm of y = {res.ynorm:.6g}")

    if mat_comp:
        A = CSROperator(pb)
        z = pb.new_vector()
        _sync(pb)
        with timed("% CSR Matvec", sync=lambda: _sync(pb)):
            if use_cg:
                cg_solve(A, pb, z, u, nreps, 0.0)
            else:
                for _ in range(nreps):
                    A.apply(u, z)
        res.znorm = pb.norm(z)
        e = z - y
        res.enorm = pb.norm(e)
        if rank0:
            printer(f"Norm of u = {res.unorm:.6g}")
            printer(f"Norm of z = {res.znorm:.6g}")
            printer(f"Norm of error = {res.enorm:.6g}")
            rel = res.enorm / res.znorm if res.znorm != 0 else float("nan")
            printer(f"Relative norm of error = {rel:.6g}")
    if hasattr(op, "close"):
        op.close()  # native runtime: release RCCL / graphs before shutdown
    return res
