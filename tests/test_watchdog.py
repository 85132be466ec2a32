"""Deadline policy of the native runtime's RCCL watchdog
(csrc/include/bdx_watchdog.h), exercised on the CPU through the host library:
a blocking call that outlives the deadline, or an asynchronous communicator
error, fires the abort once; a call inside the deadline does not."""

import ctypes

import pytest

from benchmark_dolfinx_amd.ops import native


def _run(timeout_s, busy_s, err_after_s):
    lib = native.host()
    fn = lib.bdx_watchdog_selftest
    fn.argtypes = [ctypes.c_double] * 3 + [ctypes.c_void_p, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    fire, reason = ctypes.c_double(0), ctypes.c_int(0)
    fired = fn(timeout_s, busy_s, err_after_s, ctypes.byref(fire), ctypes.byref(reason))
    return fired, fire.value, reason.value


def test_fires_after_the_deadline():
    fired, t, reason = _run(0.2, 5.0, -1)
    assert fired == 1 and reason == 1
    assert 0.2 <= t < 1.5, t  # the "hung call" returned once the abort ran, not after 5 s


def test_quiet_inside_the_deadline():
    fired, t, reason = _run(2.0, 0.1, -1)
    assert fired == 0 and reason == 0 and t < 0


def test_async_error_fires_before_the_deadline():
    fired, t, reason = _run(30.0, 5.0, 0.1)
    assert fired == 1 and reason == 2
    assert 0.1 <= t < 1.5, t


@pytest.mark.parametrize("timeout", [0.0])
def test_zero_timeout_disables_the_deadline(timeout):
    fired, _, _ = _run(timeout, 0.3, -1)
    assert fired == 0
