"""The native runtime's RCCL transport on real hardware.

RCCL refuses two ranks on one GPU, so the multi-rank loop is rehearsed with the
thread transport (test_gpu_distributed_emulated.py).  This test runs the
RCCL calls themselves -- grouped ncclSend/ncclRecv (RcclTransport::exchange),
the device-scalar ncclAllReduce, and both again inside a captured hipGraph --
on a 1-rank communicator of the box's GPU (runtime.hip: bdx_rt_rccl_selftest).
"""

import pytest
import torch

from benchmark_dolfinx_amd.ops import native
from benchmark_dolfinx_amd.ops.kernels import _stream
from benchmark_dolfinx_amd.ops.native import ptr

pytestmark = pytest.mark.gpu


def test_rccl_transport_selftest():
    lib = native.hip()
    n = 4099
    buf = torch.zeros(3 * n + 2, dtype=torch.float64, device="cuda")
    src = torch.arange(n, dtype=torch.float64, device="cuda") * 0.25 - 7.0
    buf[:n] = src
    buf[2 * n] = 3.0
    buf[2 * n + 1] = -7.25
    torch.cuda.synchronize()
    rc = lib.bdx_rt_rccl_selftest(ptr(buf), n, _stream())
    torch.cuda.synchronize()
    assert rc == 0, f"bdx_rt_rccl_selftest returned {rc}"
    assert torch.equal(buf[n:2 * n], src)            # eager grouped send/recv
    assert torch.equal(buf[2 * n + 2:], src)         # the same, replayed from a graph
    assert buf[2 * n].item() == 3.0 and buf[2 * n + 1].item() == -7.25  # 1-rank sums
