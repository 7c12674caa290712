#!/usr/bin/env python3
"""Prefill GEMM solution selection with PyTorch TunableOp (hipBLASLt + rocBLAS
solutions timed per exact shape) vs the library heuristic, on a model's prefill
GEMMs at M = the engine's token budget. Reports the tuning cost per shape and the
32-layer chain time before/after, and writes the tuned table.

    python tools/tune_prefill_gemm.py [--model llama-3-8b] [--m 8192] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipserve.config import PRESETS  # noqa: E402
from hipserve.ops import prefill_tune  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama-3-8b")
ap.add_argument("--m", type=int, default=8192)
ap.add_argument("--layers", type=int, default=8)
ap.add_argument("--out", default="gpurun_out/tunableop_prefill.csv")
ap.add_argument("--duration-ms", type=float, default=prefill_tune.TUNE_MS)
a = ap.parse_args()

mc = PRESETS[a.model]
shapes = prefill_tune.model_prefill_shapes(mc, tp=1)
dev = "cuda"
L = a.layers
W = {s: [torch.randn(*s, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(L)] for s in shapes}
X = {s: torch.randn(a.m, s[1], device=dev, dtype=torch.bfloat16) for s in shapes}


def chain():
    for i in range(L):
        for s in shapes:
            F.linear(X[s], W[s][i])


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return best / L


flops = 2 * a.m * sum(n * k for n, k in shapes)
before = timed(chain)
print(json.dumps({"shapes": shapes, "default_ms_per_layer": round(before, 4),
                  "default_PF": round(flops / before / 1e12, 3)}), flush=True)
t0 = time.time()
tuned = prefill_tune.tune(shapes, [a.m], dev, filename=a.out, duration_ms=a.duration_ms)
print(json.dumps({"tune_s": round(time.time() - t0, 2), "tuned": tuned}), flush=True)
after = timed(chain)
print(json.dumps({"tuned_ms_per_layer": round(after, 4), "tuned_PF": round(flops / after / 1e12, 3),
                  "speedup": round(before / after, 3)}), flush=True)
