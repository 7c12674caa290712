#!/usr/bin/env python3
"""Prefill GEMMs of Llama-3-8B (M = 8192) timed three ways: one weight repeated
(hot, what TunableOp measures), all 32 layers back to back (a prefill step's
weight stream), and back to back with the elementwise ops between them."""
import json
import sys

import torch
import torch.nn.functional as F

M, H, I, L = 8192, 4096, 14336, 32
dev = "cuda"
shapes = {"qkv": (6144, H), "o": (H, H), "gu": (2 * I, H), "down": (H, I)}
W = {k: [torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)] for k, (n, kk) in shapes.items()}
xs = {k: torch.randn(M, kk, device=dev, dtype=torch.bfloat16) for k, (n, kk) in shapes.items()}


def ev():
    return torch.cuda.Event(enable_timing=True)


def time_fn(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        a, b = ev(), ev()
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


res = {}
for k in shapes:  # hot: same weight 32 times
    res[f"hot_{k}_ms"] = round(time_fn(lambda: [F.linear(xs[k], W[k][0]) for _ in range(L)]) / L, 4)
for k in shapes:  # cold-ish: 32 different weights
    res[f"stream_{k}_ms"] = round(time_fn(lambda: [F.linear(xs[k], W[k][i]) for i in range(L)]) / L, 4)


def layer_chain():
    for i in range(L):
        F.linear(xs["qkv"], W["qkv"][i])
        F.linear(xs["o"], W["o"][i])
        F.linear(xs["gu"], W["gu"][i])
        F.linear(xs["down"], W["down"][i])


res["chain_per_layer_ms"] = round(time_fn(layer_chain) / L, 4)
flops = 2 * M * sum(n * kk for n, kk in shapes.values())
res["chain_PFLOPs"] = round(flops / (res["chain_per_layer_ms"] * 1e-3) / 1e15, 3)
print(json.dumps(res), flush=True)
