"""End-to-end CLI runs (the reference CI, .github/workflows/ci.yml:100-115):
serial and 2-process (gloo over torch.distributed.run, the analogue of the
CI's oversubscribed `mpirun -n 2`), checked with the golden JSON checker;
plus the bench.py output contract on the CPU platform."""

import json
import os
import subprocess
import sys

import pytest

from benchmark_dolfinx_amd.utils.check_output import check

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CI_ARGS = ["--platform=cpu", "--degree=3", "--qmode=0", "--nreps=1", "--mat_comp", "--float=64"]


def _env():
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "2"
    return env


def _run(cmd, timeout=300):
    r = subprocess.run(cmd, cwd=ROOT, env=_env(), capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _torchrun(n, port):
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}"]


def test_cli_serial_golden(tmp_path):
    js = tmp_path / "a.json"
    out = _run([sys.executable, "-m", "benchmark_dolfinx_amd", "--ndofs=1000", *CI_ARGS,
                "--json", str(js)])
    assert "Computation rate (Gdofs/s):" in out and "Relative norm of error" in out
    data = check(str(js))
    assert set(data["input"]) == {"p", "mpi_size", "ndofs_local_requested", "nreps",
                                  "scalar_size", "use_gauss", "mat_comp", "qmode", "cg"}
    assert set(data["output"]) == {"ncells_global", "ndofs_global", "mat_free_time",
                                   "u_norm", "y_norm", "z_norm", "gdof_per_second"}


@pytest.mark.parametrize("n", [2, 4])
def test_cli_multiprocess_golden(tmp_path, n):
    js = tmp_path / "b.json"
    _run(_torchrun(n, 29610 + n) + ["-m", "benchmark_dolfinx_amd", f"--ndofs={1000 // n}",
                                    *CI_ARGS, "--json", str(js)])
    data = check(str(js))
    assert data["input"]["mpi_size"] == n


def test_cli_multiprocess_cg_mat_comp(tmp_path):
    """CG on the matrix-free operator vs CG on the assembled CSR, 2 processes."""
    js = tmp_path / "c.json"
    _run(_torchrun(2, 29631) + ["-m", "benchmark_dolfinx_amd", "--platform=cpu",
                                "--ndofs_global=20000", "--degree=2", "--qmode=1", "--cg",
                                "--nreps=10", "--mat_comp", "--geom_perturb_fact=0.1",
                                "--json", str(js)])
    out = json.load(open(js))["output"]
    assert abs(out["y_norm"] - out["z_norm"]) < 1e-10 * out["z_norm"]


def test_cli_option_validation():
    r = subprocess.run([sys.executable, "-m", "benchmark_dolfinx_amd", "--ndofs=10",
                        "--ndofs_global=10"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True)
    assert r.returncode != 0 and "Conflicting" in (r.stdout + r.stderr)
    r = subprocess.run([sys.executable, "-m", "benchmark_dolfinx_amd", "--float=16"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True)
    assert r.returncode != 0


def test_cli_unknown_options_pass_through(tmp_path):
    # spdlog-style level arguments are accepted (allow_unregistered)
    _run([sys.executable, "-m", "benchmark_dolfinx_amd", "--ndofs=1000", *CI_ARGS,
          "SPDLOG_LEVEL=info"])


def test_bench_contract_cpu():
    out = _run([sys.executable, "bench.py", "--platform", "cpu", "--dofs-per-gpu", "20000",
                "--steps", "2", "--warmup", "1"])
    line = json.loads(out.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line, k
    assert line["n_gpus"] == 1 and line["steps"] == 2 and line["scaling"] == "weak"
    for k in ("model", "global_batch", "seq_len", "parallelism"):
        assert k in line["config"]


def test_bench_contract_cpu_2ranks():
    out = _run(_torchrun(2, 29641) + ["bench.py", "--platform", "cpu", "--gpus", "2",
                                      "--dofs-per-gpu", "10000", "--steps", "2",
                                      "--warmup", "1"])
    line = json.loads([s for s in out.strip().splitlines() if s.startswith("{")][-1])
    assert line["n_gpus"] == 2
