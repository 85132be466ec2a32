"""In-tree build of the native libraries.

* ``libbdx_host.so``: C++17 host runtime (g++, -O3, OpenMP): CPU operator,
  CSR assembly, SpMV, interpolation.
* ``libbdx_hip.so``: HIP kernels for gfx950 only (hipcc
  --offload-arch=gfx950, -munsafe-fp-atomics like the reference's
  src/CMakeLists.txt:53-61).  Translation units are compiled in parallel and
  linked into one shared object.

Both land next to this file so they travel with the repo snapshot to the
GPU box (they are git-ignored).  Nothing is written under ~/.cache.

Usage: ``python -m benchmark_dolfinx_amd.ops.build [--host] [--hip] [-j N]``
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
PKG = HERE.parent
CSRC = PKG / "csrc"
HOST_SO = HERE / "libbdx_host.so"
HIP_SO = HERE / "libbdx_hip.so"
OBJ_DIR = PKG / "csrc" / "build"

HIP_ARCH = os.environ.get("BDX_HIP_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _sources(sub: str, ext: str, csrc: Path = CSRC) -> list[Path]:
    return sorted((csrc / sub).glob(f"*{ext}"))


def _headers(csrc: Path = CSRC) -> list[Path]:
    return sorted((csrc / "include").glob("*.h")) + sorted((csrc / "hip").glob("*.h"))


def _digest(paths: list[Path], extra: str = "") -> str:
    h = hashlib.sha1(extra.encode())
    for p in paths:
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()


def _up_to_date(target: Path, digest: str) -> bool:
    stamp = target.with_suffix(target.suffix + ".sha1")
    return target.exists() and stamp.exists() and stamp.read_text().strip() == digest


def _stamp(target: Path, digest: str) -> None:
    target.with_suffix(target.suffix + ".sha1").write_text(digest + "\n")


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build failed: {cmd[0]} ... {cmd[-1]}")


HOST_SAN_SO = HERE / "libbdx_host_san.so"
SAN_FLAGS = ["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
             "-fno-sanitize-recover=undefined"]


def build_host(force: bool = False, sanitize: bool = False) -> Path:
    """libbdx_host.so; with `sanitize`, libbdx_host_san.so built with
    AddressSanitizer + UndefinedBehaviorSanitizer (host code only: load it with
    BDX_HOST_LIB and LD_PRELOAD=libasan.so, see tests/test_host_sanitizers.py)."""
    srcs = _sources("host", ".cpp")
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-march=x86-64-v2",
             "-Wall", "-Wno-unknown-pragmas"]
    out = HOST_SO
    if sanitize:
        flags = [f for f in flags if f != "-O3"] + SAN_FLAGS
        out = HOST_SAN_SO
    digest = _digest(srcs + _headers(), " ".join(flags))
    if not force and _up_to_date(out, digest):
        return out
    cxx = shutil.which("g++") or "c++"
    tmp = out.with_suffix(".so.tmp")
    _run([cxx, *flags, "-I", str(CSRC / "include"), *map(str, srcs), "-o", str(tmp)])
    os.replace(tmp, out)
    _stamp(out, digest)
    return out


def hip_flags(csrc: Path = CSRC) -> list[str]:
    return ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={HIP_ARCH}",
            "-munsafe-fp-atomics", "-ffp-contract=fast", "-Wno-unused-result",
            # MFMA accumulators in VGPRs (unified register file): the AGPR form
            # pushed the Q6 fused3 CG instance over 256 registers (1 wave / SIMD)
            "-mllvm", "-amdgpu-mfma-vgpr-form",
            "-I", str(csrc / "include"), "-I", str(csrc / "hip")]


def build_hip(force: bool = False, jobs: int | None = None,
              extra_flags: list[str] | None = None, variant: str = "",
              only: list[str] | None = None, csrc: Path | None = None) -> Path:
    """Build libbdx_hip.so (or, with `variant`, libbdx_hip_<variant>.so with
    `extra_flags` appended: used for A/B kernel experiments on the GPU box).
    `only`: for a variant, the operator TUs (lap_fused*_*.hip stems) to keep;
    every other operator TU is left out to save compile time.  `csrc`: for a
    variant, an alternative source tree (an experimental copy of csrc/)."""
    if csrc is None or not variant:
        csrc = CSRC
    csrc = Path(csrc)
    srcs = _sources("hip", ".hip", csrc)
    if only:
        srcs = [p for p in srcs if not p.stem.startswith("lap_fused") or p.stem in only]
    flags = hip_flags(csrc) + list(extra_flags or [])
    out_so = HIP_SO if not variant else HERE / f"libbdx_hip_{variant}.so"
    obj_dir = OBJ_DIR if not variant else OBJ_DIR / variant
    digest = _digest(srcs + _headers(csrc), " ".join(flags))
    if not force and _up_to_date(out_so, digest):
        return out_so
    if not Path(HIPCC).exists():
        raise RuntimeError(f"hipcc not found at {HIPCC}")
    obj_dir.mkdir(parents=True, exist_ok=True)
    jobs = jobs or min(8, os.cpu_count() or 4, max(1, len(srcs)))

    def compile_one(src: Path) -> Path:
        obj = obj_dir / (src.stem + ".o")
        odig = _digest([src] + _headers(csrc), " ".join(flags))
        if not force and _up_to_date(obj, odig):
            return obj
        _run([HIPCC, *flags, "-c", str(src), "-o", str(obj)])
        _stamp(obj, odig)
        return obj

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = out_so.with_suffix(".so.tmp")
    # RCCL: resolved at load time against the librccl.so.1 torch already
    # loaded (same SONAME), so the process holds one RCCL
    _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={HIP_ARCH}", *map(str, objs),
          "-L/opt/rocm/lib", "-lrccl", "-o", str(tmp)])
    os.replace(tmp, out_so)
    _stamp(out_so, digest)
    return out_so


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", action="store_true")
    ap.add_argument("--hip", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("--variant", action="append", default=[],
                    help="NAME=FLAGS: also build libbdx_hip_NAME.so with extra hipcc flags")
    ap.add_argument("--sanitize", action="store_true",
                    help="also build libbdx_host_san.so (ASan + UBSan host library)")
    ap.add_argument("--only", default="",
                    help="comma-separated operator TU stems to keep in variant builds")
    ap.add_argument("--csrc", default=None,
                    help="variant builds: alternative source tree (a copy of csrc/)")
    a = ap.parse_args(argv)
    only = [x for x in a.only.split(",") if x] or None
    for v in a.variant:
        name, _, fl = v.partition("=")
        print("built", build_hip(a.force, a.jobs, fl.split(), name, only, a.csrc))
    if a.variant and not (a.host or a.hip):
        return 0
    if a.sanitize:
        print("built", build_host(a.force, sanitize=True))
    both = not (a.host or a.hip)
    if a.host or both:
        print("built", build_host(a.force))
    if a.hip or both:
        print("built", build_hip(a.force, a.jobs))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
