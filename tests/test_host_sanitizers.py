"""Host-code sanitizers (SURVEY §5 race/sanitizer row): the C++ host library
(CPU operator, CSR assembly + SpMV, RHS interpolation) rebuilt with
AddressSanitizer + UndefinedBehaviorSanitizer (`ops/build.py --sanitize`),
then the CPU operator suite and a CLI `--mat_comp` run (CSR assembly, 2-rank
gloo) execute against it in subprocesses.  Any ASan/UBSan report aborts the
child (halt_on_error) and fails the test.  GPU code is not sanitized (no GPU
ASan on this pool); the HIP kernels have BDX_DEBUG device-side index checks
instead (csrc/hip/bdx_common.h)."""

import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _san_env():
    from benchmark_dolfinx_amd.ops.build import build_host
    lib = build_host(sanitize=True)
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++ to locate libasan")
    asan = subprocess.run([gxx, "-print-file-name=libasan.so"], capture_output=True,
                          text=True).stdout.strip()
    if not os.path.isabs(asan) or not os.path.exists(asan):
        pytest.skip("libasan.so not found")
    env = dict(os.environ)
    env.update(LD_PRELOAD=asan, BDX_HOST_LIB=str(lib), OMP_NUM_THREADS="2",
               ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PYTHONPATH=ROOT + os.pathsep + env.get("PYTHONPATH", ""))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    return env, str(lib)


def _run(args, env, timeout=600):
    r = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert "AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    return out


def test_sanitized_host_library_is_the_one_loaded():
    env, lib = _san_env()
    out = _run([sys.executable, "-c", "from benchmark_dolfinx_amd.ops import native; "
                "native.host(); print(native.loaded_libraries())"], env, 120)
    assert lib in out


def test_cpu_operator_suite_under_asan_ubsan():
    env, _ = _san_env()
    _run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
          "tests/test_cpu_operator.py"], env)


def test_cli_mat_comp_two_ranks_under_asan_ubsan(tmp_path):
    env, _ = _san_env()
    _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
          "--master-addr=127.0.0.1", "--master-port=29731", "-m", "benchmark_dolfinx_amd",
          "--platform=cpu", "--ndofs=3000", "--degree=3", "--qmode=1", "--nreps=2",
          "--mat_comp", "--geom_perturb_fact=0.1", f"--json={tmp_path / 'o.json'}"], env)
