#!/usr/bin/env python3
"""Workload for PMC passes over the prefill attention kernel (scripts/pg_pmc.sh with
PMC_PY=tools/attn_pmc.py PG_SHAPE=<S>): 8,192 query tokens as 8192/S causal
sequences of S tokens (Llama-3-8B heads: 32 q / 8 kv, D 128), a few launches after a
warm-up — 1K-token prompts (the headline's prefill) against 8K / 32K ones."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipserve.ops import KernelOps  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    ops = KernelOps()
    D, bs, nq, nkv = 128, 16, 32, 8
    nseq = max(1, 8192 // S)
    dev = "cuda"
    mb = S // bs
    kc = torch.randn(nseq * mb, nkv, bs, D, device=dev, dtype=torch.bfloat16)
    vc = torch.randn(nseq * mb, nkv, D, bs, device=dev, dtype=torch.bfloat16)
    bt = torch.arange(nseq * mb, device=dev).int().view(nseq, mb)
    cu = torch.arange(0, (nseq + 1) * S, S, device=dev, dtype=torch.int32)
    ctx = torch.full((nseq,), S, device=dev, dtype=torch.int32)
    tiles = torch.tensor(sorted(((s, r) for s in range(nseq) for r in range(0, S, 128)), key=lambda t: -t[1]),
                         device=dev, dtype=torch.int32)
    q = torch.randn(nseq * S, (nq + 2 * nkv) * D, device=dev, dtype=torch.bfloat16)
    out = torch.empty(nseq * S, nq * D, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        ops.prefill_attention(out, q, kc, vc, bt, cu, ctx, tiles, nq, nkv, 1 / math.sqrt(D))
    torch.cuda.synchronize()
    print("ok", S, nseq)


if __name__ == "__main__":
    main()
