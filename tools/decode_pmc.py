#!/usr/bin/env python3
"""Workload for PMC passes over the paged decode kernel (scripts/pg_pmc.sh with
PMC_PY=tools/decode_pmc.py PG_SHAPE=<ctx>): Llama-3-8B heads (32 q / 8 kv, D 128),
B = 64 sequences of <ctx> keys, one partition per (sequence, kv head), a bf16 and an
e4m3 cache (--kv-cache-dtype fp8), each launched over 4 rotated cache copies so every
call streams cold K / V."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipserve.ops import KernelOps  # noqa: E402


def main():
    ctx = int(sys.argv[1]) if len(sys.argv) > 1 else 1152
    ops = KernelOps()
    D, bs, nq, nkv, B, part = 128, 16, 32, 8, 64, 2048
    dev = "cuda"
    mb = math.ceil(ctx / bs) + 1
    bt = torch.randperm(B * mb, device=dev).int().view(B, mb)
    cl = torch.full((B,), ctx, device=dev, dtype=torch.int32)
    q = torch.randn(B, (nq + 2 * nkv) * D, device=dev, dtype=torch.bfloat16)
    mp = math.ceil(mb * bs / part)
    to = torch.empty(B, nq, mp, D, device=dev)
    tm = torch.empty(B, nq, mp, 2, device=dev)
    out = torch.empty(B, nq * D, device=dev, dtype=torch.bfloat16)
    for kvt in (torch.bfloat16, torch.float8_e4m3fn):
        kcs = [torch.randn(B * mb, nkv, bs, D, device=dev).to(kvt) for _ in range(4)]
        vcs = [torch.randn(B * mb, nkv, D, bs, device=dev).to(kvt) for _ in range(4)]
        for i in range(8):
            ops.paged_decode(out, q, kcs[i % 4], vcs[i % 4], bt, cl, to, tm, nq, nkv, part, 1 / math.sqrt(D))
        torch.cuda.synchronize()
        del kcs, vcs
    print("ok", ctx)


if __name__ == "__main__":
    main()
