#!/usr/bin/env python3
"""Repeatability check of the hand-written prefill GEMM variants: the same operands
N times per variant, every result compared with the first run and with an fp32
reference; prints mismatch counts per run. A race in the LDS-DMA pipeline shows up
as run-to-run differences.  usage: python tools/pg_race.py [reps] [M N K]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hipserve.ops import load_library

load_library()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
M, N, K = (int(a) for a in sys.argv[2:5]) if len(sys.argv) >= 5 else (8192, 512, 4096)
g = torch.Generator(device="cuda").manual_seed(M + N + K)
x = ((torch.rand(M, K, device="cuda", generator=g) * 2 - 1)).to(torch.bfloat16)
w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
want = x.float() @ w.float().t()
tol = 1e-2 * want.abs().max().item()
for v in (1, 2):
    first, bad_runs, diff_runs = None, 0, 0
    for r in range(reps):
        out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        torch.ops.hipserve.prefill_gemm(out, x, w, 0, v)
        torch.cuda.synchronize()
        nbad = int(((out.float() - want).abs() > tol).sum())
        bad_runs += nbad > 0
        if first is None:
            first = out
        elif not torch.equal(out, first):
            diff_runs += 1
        if nbad:
            idx = ((out.float() - want).abs() > tol).nonzero()[:4].tolist()
            print(f"variant {v} run {r}: {nbad} wrong, e.g. {idx}", flush=True)
    print(f"variant {v}: {bad_runs}/{reps} runs with wrong elements, {diff_runs} runs differ from run 0", flush=True)
