"""Locate fused-kernel fp32 errors vs the CPU operator (GPU box)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from benchmark_dolfinx_amd.models.fused import FusedLaplacianGPU
from benchmark_dolfinx_amd.models.poisson import MatFreeLaplacianCPU, MatFreeLaplacianGPU, PoissonProblem
from benchmark_dolfinx_amd.parallel.comm import Comm
for nc, P, qm, pert in [((5, 4, 7), 3, 1, 0.2), ((5, 4, 7), 3, 1, 0.0), ((2, 2, 5), 3, 1, 0.0), ((2, 2, 2), 3, 1, 0.0), ((2, 3, 3), 6, 1, 0.0)]:
    for dt in (torch.float32, torch.float64):
        gpu = PoissonProblem(Comm(), nc, P, qm, False, dt, "gpu", pert)
        cpu = PoissonProblem(Comm(), nc, P, qm, False, torch.float64, "cpu", pert)
        u64 = torch.from_numpy(np.random.default_rng(3).standard_normal(cpu.lat.shape))
        yc = cpu.new_vector(); MatFreeLaplacianCPU(cpu).apply(u64, yc)
        for geom in ("otf", "stored"):
            yg = torch.zeros(gpu.lat.shape, dtype=dt, device=gpu.device)
            FusedLaplacianGPU(gpu, geom).apply(u64.to(gpu.device, dt), yg)
            yv = gpu.new_vector(); MatFreeLaplacianGPU(gpu, geom).apply(u64.to(gpu.device, dt), yv)
            o = cpu.owned
            d = (o(yg.double().cpu()) - o(yc)).abs()
            dv = (o(yv.double().cpu()) - o(yc)).abs()
            idx = np.argwhere(d.numpy() > 1e-3 * yc.abs().max().item())
            print(nc, P, dt, geom, "fused err %.3e v1 err %.3e" % (d.max().item(), dv.max().item()), "bad", len(idx), idx[:6].tolist())
