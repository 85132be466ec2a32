"""`bench_dolfinx` command line (same options, console lines and JSON as the
reference's src/main.cpp:136-320).

Run:  python -m benchmark_dolfinx_amd [options]
      torchrun --nproc-per-node N -m benchmark_dolfinx_amd [options]

Reference options (src/main.cpp:144-183): --platform, --float, --ndofs,
--ndofs_global, --qmode, --cg, --nreps, --degree, --mat_comp,
--geom_perturb_fact, --use_gauss, --json.  Unknown options are accepted
(like `allow_unregistered`, used for `SPDLOG_LEVEL=...`).

MI355X extensions (additive): --kernel {auto,fused5,fused3,fused2,
fused,v1,dofmap}, --geometry {auto,otf,otf-general,stored}, --kappa {constant,random},
--warmup N (untimed repetitions before the timed loop).
The JSON gains an additive "mi355x" object; the reference keys are
unchanged.
"""

from __future__ import annotations

import argparse
import json
import os
import sys

BANNER = """DOLFINx benchmark (MI355X-native)
-----------------

  Finite Element Operator Action Benchmark which computes
  the Laplacian operator on a cube mesh of hexahedral elements.
"""


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="bench_dolfinx", description=BANNER,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--platform", default=None, help="Compute platform (cpu or gpu)")
    ap.add_argument("--float", type=int, default=64, help="Float size (bits). 32 or 64.")
    ap.add_argument("--ndofs", type=int, default=None,
                    help="Number of degrees-of-freedom per process (default 1000)")
    ap.add_argument("--ndofs_global", type=int, default=None,
                    help="Number of global degrees-of-freedom")
    ap.add_argument("--qmode", type=int, default=1,
                    help="Quadrature mode (0 or 1): qmode=0 has P+1 points in each "
                         "direction, qmode=1 has P+2 points in each direction.")
    ap.add_argument("--cg", action="store_true",
                    help="Do CG iterations, rather than simple operator action")
    ap.add_argument("--nreps", type=int, default=1000, help="Number of repetitions")
    ap.add_argument("--degree", type=int, default=3, help='Polynomial degree "P" (1-7)')
    ap.add_argument("--mat_comp", action="store_true",
                    help="Compare result to matrix operator (slow with large ndofs)")
    ap.add_argument("--geom_perturb_fact", type=float, default=0.0,
                    help="Randomly perturb the geometry (useful to check correctness)")
    ap.add_argument("--use_gauss", action="store_true",
                    help="Use Gauss quadrature rather than GLL quadrature")
    ap.add_argument("--json", default="", help="Filename for JSON output")
    # MI355X extensions
    ap.add_argument("--kernel", default="auto",
                    choices=["auto", "fused5", "fused3", "fused2", "fused", "v1", "dofmap"],
                    help="GPU operator kernel: fused structured kernel, the generic v1, or the "
                         "unstructured dofmap data model")
    ap.add_argument("--geometry", default="auto", choices=["auto", "otf", "otf-general", "stored"],
                    help="Geometry factors on the fly (otf: constant-Jacobian fast path for "
                         "parallelepiped cells; otf-general: always the trilinear path) or "
                         "precomputed (stored, the reference's layout)")
    ap.add_argument("--kappa", default="constant", choices=["constant", "random"],
                    help="Diffusion coefficient: the reference's constant 2.0, or a random "
                         "per-cell field U(1, 3) (partition-invariant)")
    ap.add_argument("--warmup", type=int, default=0,
                    help="Untimed repetitions before the timed loop")
    return ap


def parse_args(argv=None):
    ap = build_parser()
    args, unknown = ap.parse_known_args(argv)
    if args.ndofs is not None and args.ndofs_global is not None:
        raise SystemExit("error: Conflicting options 'ndofs' and 'ndofs_global'")
    if args.float not in (32, 64):
        raise SystemExit("error: Invalid float size. Must be 32 or 64.")
    if args.qmode > 1 or args.qmode < 0:
        raise SystemExit("error: Invalid qmode.")
    return args, unknown


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    args, unknown = parse_args(argv)

    import torch

    from .fem.mesh import compute_mesh_size
    from .parallel.comm import finalize, init_distributed
    from .utils.log import init_logging
    from .utils.timing import list_timings

    platform = args.platform
    if platform is None:
        platform = "gpu" if torch.cuda.is_available() else "cpu"
    if platform not in ("cpu", "gpu"):
        raise RuntimeError("Invalid platform: " + platform)
    comm = init_distributed(platform)
    log = init_logging(unknown, comm.rank)
    size = comm.size
    ndofs = args.ndofs if args.ndofs is not None else 1000
    if args.ndofs_global is None:
        ndofs_global = ndofs * size
    else:
        ndofs_global = args.ndofs_global
        ndofs = ndofs_global // size

    rank0 = comm.rank == 0
    if rank0:
        if platform == "gpu":
            from .ops.kernels import device_info
            print(device_info(torch.cuda.current_device()), end="")
        print("-----------------------------------")
        print(f"Platform: {platform}")
        print(f"Polynomial degree : {args.degree}")
        print(f"Number of ranks : {size}")
        print(f"Requested number of local DoFs : {ndofs}")
        print(f"Number of repetitions : {args.nreps}")
        print(f"Scalar Type: {args.float}")
        print(f"Use Gauss-Jacobi: {int(args.use_gauss)}")
        print(f"Compare to matrix: {int(args.mat_comp)}")
        print("-----------------------------------", flush=True)

    in_root = {"p": args.degree, "mpi_size": size, "ndofs_local_requested": ndofs,
               "nreps": args.nreps, "scalar_size": args.float, "use_gauss": args.use_gauss,
               "mat_comp": args.mat_comp, "qmode": args.qmode, "cg": args.cg}
    nx = compute_mesh_size(ndofs_global, args.degree)
    log.info("Mesh cells in each direction: %s", nx)
    out_root, extra = run_benchmark(comm, nx, args, platform)
    if rank0 and args.json:
        root = {"input": in_root, "output": out_root, "mi355x": extra}
        print(f"*** Writing output to:       {args.json}")
        print(f"*** Writing output to (abs): {os.path.abspath(args.json)}")
        with open(args.json, "w") as fh:
            fh.write(json.dumps(root) + "\n")
    elif rank0:
        print(f"*** Empty file: {args.json}")
    table = list_timings(comm)
    if rank0:
        print(table, flush=True)
    finalize()
    return 0


def _device_name() -> str:
    import torch

    from .ops.kernels import device_name
    return device_name(torch.cuda.current_device())


def _build_flags() -> dict:
    from .ops.native import build_flags
    return build_flags()


def run_benchmark(comm, nx, args, platform):
    import torch

    from .driver import laplace_action
    from .models.poisson import PoissonProblem

    dtype = torch.float64 if args.float == 64 else torch.float32
    pb = PoissonProblem(comm, nx, args.degree, args.qmode, args.use_gauss, dtype,
                        platform, args.geom_perturb_fact, args.kappa)
    res = laplace_action(pb, args.nreps, args.cg, args.mat_comp, kernel=args.kernel,
                         geometry=args.geometry, warmup=args.warmup)
    t = res.mat_free_time
    gdofs = pb.ndofs_global * args.nreps / (1e9 * t) if t > 0 else 0.0
    out = {"ncells_global": pb.ncells_global, "ndofs_global": pb.ndofs_global,
           "mat_free_time": t, "u_norm": res.unorm, "y_norm": res.ynorm,
           "z_norm": res.znorm, "gdof_per_second": gdofs}
    extra = {"gdof_per_second_per_gpu": gdofs / comm.size, "mesh": list(nx),
             "partition": list(pb.lat.pgrid), "e_norm": res.enorm,
             "device": _device_name() if platform == "gpu" else "cpu",
             "build_flags": _build_flags() if platform == "gpu" else None,
             **res.extra}
    return out, extra


if __name__ == "__main__":
    raise SystemExit(main())
