#!/usr/bin/env python3
"""HBM streaming bandwidth of simple torch ops on the box (reference points for
the r-update pass: 2 reads + 1 write of 300 M / 500 M doubles)."""
import torch


def bw(fn, nbytes, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return ms, nbytes / (ms * 1e-3) / 1e12


for n in (300_000_000, 500_000_000):
    r = torch.rand(n, dtype=torch.float64, device="cuda")
    y = torch.rand(n, dtype=torch.float64, device="cuda")
    z = torch.empty_like(r)
    b = 8 * n
    ms, tb = bw(lambda: z.copy_(r), 2 * b)
    print(f"n={n}: copy            {ms:7.3f} ms  {tb:5.2f} TB/s")
    ms, tb = bw(lambda: r.add_(y, alpha=-1e-9), 3 * b)
    print(f"n={n}: r += a*y (2R1W) {ms:7.3f} ms  {tb:5.2f} TB/s")
    ms, tb = bw(lambda: torch.dot(r, y), 2 * b)
    print(f"n={n}: dot (2R)        {ms:7.3f} ms  {tb:5.2f} TB/s")
    del r, y, z
    torch.cuda.empty_cache()
