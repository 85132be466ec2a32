"""Race detection by determinism: the structured kernels are
atomic-free with fixed-order reductions, so repeated applies and repeated CG
solves (native runtime, hipGraph replay, 1 and 4 threaded ranks) must be
bitwise identical.  The atomic-scatter kernels (v1 -- also the RHS mass
assembly -- and dofmap, like the reference) are reproducible to rounding
only, which is asserted as such."""

import numpy as np
import pytest
import torch

from benchmark_dolfinx_amd.driver import make_operator
from benchmark_dolfinx_amd.models.poisson import PoissonProblem
from benchmark_dolfinx_amd.parallel.comm import Comm, run_threaded
from benchmark_dolfinx_amd.solvers.cg import DeviceCG

pytestmark = pytest.mark.gpu

KERNELS = [("fused5", 3, 0.0), ("fused5", 6, 0.0), ("fused5", 4, 0.0), ("fused3", 3, 0.15),
           ("fused2", 3, 0.15)]


@pytest.mark.parametrize("kernel,P,pert", KERNELS)
def test_apply_is_bitwise_reproducible(kernel, P, pert):
    pb = PoissonProblem(Comm(), (5, 9, 11), P, 1, False, torch.float64, "gpu", pert, "random")
    op = make_operator(pb, kernel)
    assert getattr(op, "name", "") == kernel
    rng = np.random.default_rng(3)
    u = torch.from_numpy(rng.standard_normal(pb.lat.shape)).to(pb.device)
    outs = []
    for _ in range(3):
        y = torch.full(pb.lat.shape, float("nan"), dtype=torch.float64, device=pb.device)
        op.apply(u, y)
        torch.cuda.synchronize()
        outs.append(pb.owned(y).clone())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    if hasattr(op, "close"):
        op.close()


def _cg(comm, kernel, P, nits):
    pb = PoissonProblem(comm, (6, 10, 12), P, 1, False, torch.float64, "gpu", 0.0, "random")
    # a partition-invariant right-hand side from the global dof index (the
    # assembled RHS uses the atomic v1 mass kernel, reproducible to rounding only)
    gi = pb.lat.global_indices()
    host = np.zeros(pb.lat.shape)
    host[:, :, :gi.shape[2]] = np.sin(0.37 * gi) + 0.5
    u = torch.from_numpy(host).to(pb.device)
    x = pb.new_vector()
    op = make_operator(pb, kernel)
    cg = DeviceCG(pb)
    cg.solve(op, x, u, nits)
    cg.wait()
    xn = pb.norm(x)
    if hasattr(op, "close"):
        op.close()
    return xn


@pytest.mark.parametrize("kernel,P", [("fused5", 3), ("fused5", 6), ("fused3", 3)])
def test_cg_is_bitwise_reproducible(kernel, P):
    a = run_threaded(1, _cg, kernel, P, 25)[0]
    b = run_threaded(1, _cg, kernel, P, 25)[0]
    assert a == b
    r4a = run_threaded(4, _cg, kernel, P, 25)
    r4b = run_threaded(4, _cg, kernel, P, 25)
    assert r4a == r4b  # same partition: identical to the last bit


def test_atomic_operator_reproducible_to_rounding():
    pb = PoissonProblem(Comm(), (5, 6, 7), 3, 1, False, torch.float64, "gpu", 0.1)
    op = make_operator(pb, "dofmap")
    u = torch.from_numpy(np.random.default_rng(4).standard_normal(pb.lat.shape)).to(pb.device)
    y1, y2 = pb.new_vector(), pb.new_vector()
    op.apply(u, y1)
    op.apply(u, y2)
    d = (pb.owned(y1) - pb.owned(y2)).abs().max().item()
    assert d <= 1e-13 * pb.owned(y1).abs().max().item()
