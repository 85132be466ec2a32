"""bench.py times its one-rank variants in fresh child processes
(`_measure_isolated`): the child is this script with the variant's options,
its JSON line is parsed back into the variant record, and a failing child
surfaces as an error record, not a hang.  Run here on the CPU platform (the
GPU path is the same code)."""

import argparse
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _args(**kw):
    a = argparse.Namespace(platform="cpu", dofs_per_gpu=24000, mesh=None)
    a.__dict__.update(kw)
    return a


def test_isolated_variant_matches_in_process(monkeypatch):
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    logs = []
    rec = bench._measure_isolated(_args(), "q3", 3, 1, kappa="random", perturb=0.1,
                                  log=logs.append)
    assert rec["isolated_process"] is True
    assert rec["steps"] == 3 and rec["warmup"] == 1
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    assert rec["kappa"] == "random" and rec["geom_perturb_fact"] == 0.1
    assert any("(child)" in m for m in logs)
    # the same problem in this process: the same iterate (deterministic CG)
    from benchmark_dolfinx_amd.parallel.comm import Comm
    a = bench.parse_args(["--platform", "cpu", "--dofs-per-gpu", "24000"])
    ref = bench._measure(Comm(), a, "q3", 3, 1, kappa="random", perturb=0.1)
    assert abs(rec["y_norm"] - ref["y_norm"]) <= 1e-12 * abs(ref["y_norm"])


def test_isolated_variant_failure_is_an_error(monkeypatch):
    monkeypatch.setenv("BDX_BENCH_FAIL_MEASURE", "q3")
    with pytest.raises(RuntimeError, match="isolated q3 measurement"):
        bench._measure_isolated(_args(), "q3", 2, 1)
