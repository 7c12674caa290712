#!/usr/bin/env python3
"""Run the sampler a few times for a rocprofv3 per-kernel breakdown."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from hipserve.ops import KernelOps  # noqa: E402

ops = KernelOps()
V, B = 128256, int(sys.argv[1]) if len(sys.argv) > 1 else 64
logits = (torch.randn(B, V, device="cuda") * 3).to(torch.bfloat16)
tok = torch.empty(B, dtype=torch.long, device="cuda")
lp = torch.empty(B, device="cuda")
for t, k, p in [(0.8, 0, 0.95), (0.8, 0, 1.0)]:
    temp = torch.full((B,), t, device="cuda")
    tk = torch.full((B,), k, dtype=torch.int32, device="cuda")
    tp = torch.full((B,), p, device="cuda")
    seeds = torch.arange(B, device="cuda")
    steps = torch.zeros(B, dtype=torch.long, device="cuda")
    for _ in range(10):
        ops.sample(tok, lp, logits, temp, tk, tp, seeds, steps)
torch.cuda.synchronize()
print("done")
