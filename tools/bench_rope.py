"""Prefill RoPE + KV-cache write (rope_cache tile kernel) at an 8K-token chunk:
block-aligned slots (the 16-byte V^T store path) vs a chunk starting mid-block
(2-byte V^T stores), Llama-3-8B and Llama-3-70B head shapes.

usage: python tools/bench_rope.py [--T 8192]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hipserve.ops import get_ops
from hipserve.ops import reference as ref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, nargs="+", default=[8192])
    a = ap.parse_args()
    ops = get_ops("cuda")
    dev = "cuda"
    D, bs = 128, 16
    for T, (name, nq, nkv) in [(T, m) for T in a.T for m in (("llama-3-8b", 32, 8), ("llama-3-70b", 64, 8),
                                                               ("gemma-3-27b", 32, 16))]:
        qkv = torch.randn(T, (nq + 2 * nkv) * D, device=dev, dtype=torch.bfloat16)
        pos = torch.arange(T, device=dev)
        cs = ref.rope_cos_sin(D, T + 64, 500000.0).to(dev)
        nblk = T // bs + 4
        kc = torch.zeros(nblk, nkv, bs, D, device=dev, dtype=torch.bfloat16)
        vc = torch.zeros(nblk, nkv, D, bs, device=dev, dtype=torch.bfloat16)
        moved = T * ((nq + nkv) * D * 2 + nkv * D) * 2  # q,k read + write, v read + write
        for layout, first in (("aligned", bs), ("mid-block", 5)):
            slots = torch.arange(T, device=dev) + first
            for _ in range(3):
                ops.rope_cache(qkv, pos, slots, cs, kc, vc, nq, nkv, D, 0)
            torch.cuda.synchronize()
            n = 20
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(n):
                ops.rope_cache(qkv, pos, slots, cs, kc, vc, nq, nkv, D, 0)
            e1.record()
            e1.synchronize()
            us = e0.elapsed_time(e1) * 1000 / n
            print(json.dumps({"model": name, "T": T, "slots": layout, "tile": os.environ.get("HIPSERVE_ROPE_TILE", "1"),
                              "us": round(us, 1),
                              "TB_s": round(moved / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
