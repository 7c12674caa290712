#!/usr/bin/env python3
"""rope_cache (RoPE + paged KV write) at a prefill chunk: device us per call.
HIPSERVE_ROPE_TILE=0 selects the per-token kernel for an A/B.

    python tools/bench_rope.py [--T 8192]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipserve.ops import KernelOps  # noqa: E402
from hipserve.ops import reference as ref  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=8192)
    a = ap.parse_args()
    ops = KernelOps()
    dev = torch.device("cuda", 0)
    T, nq, nkv, D, bs = a.T, 32, 8, 128, 16
    qkv = torch.randn(T, (nq + 2 * nkv) * D, device=dev, dtype=torch.bfloat16)
    pos = torch.arange(T, device=dev) % 1024
    nb = T // bs + 8
    slots = torch.arange(T, device=dev)  # 8 sequences x 1024 tokens, block-contiguous
    kc = torch.zeros(nb, nkv, bs, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(nb, nkv, D, bs, device=dev, dtype=torch.bfloat16)
    cs = ref.rope_cos_sin(D, 4096, 500000.0).to(dev)
    for _ in range(3):
        ops.rope_cache(qkv, pos, slots, cs, kc, vc, nq, nkv, D, 0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.rope_cache(qkv, pos, slots, cs, kc, vc, nq, nkv, D, 0)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / 20
    byts = T * ((nq + nkv) * D * 2 * 2 + nkv * D * 2 * 2)
    print(json.dumps({"op": "rope_cache", "T": T, "tile": os.environ.get("HIPSERVE_ROPE_TILE", "1"),
                      "us": round(us, 1), "TBps": round(byts / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
