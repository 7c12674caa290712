#!/usr/bin/env python3
"""FP8 decode GEMM A/B at decode batch sizes: the W8A16 v2 kernel (gguf_mfma.hip,
e4m3 -> f16 in VALU) vs the W8A8 kernel (fp8_decode.hip, scaled FP8 MFMA), fp32
partials for the fused epilogues, Gemma-3-27B projection shapes by default. Timed in
hipGraphs (the decode step's launch mode); one JSON line per (proj, M, kernel).
usage: python tools/bench_fp8_decode.py [--model gemma27b|llama8b] [--m 1 16 64]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from hipserve.ops import load_library, pgemm, quant as Q

SHAPES = {"gemma27b": {"qkv": ([4096, 2048, 2048], 5376), "o": ([5376], 4096), "gate_up": ([21504, 21504], 5376),
                       "down": ([5376], 21504)},
          "llama8b": {"qkv": ([4096, 1024, 1024], 4096), "o": ([4096], 4096), "gate_up": ([14336, 14336], 4096),
                      "down": ([4096], 14336)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gemma27b", choices=sorted(SHAPES))
    ap.add_argument("--m", type=int, nargs="+", default=[1, 16, 64])
    a = ap.parse_args()
    load_library()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (rows, K) in SHAPES[a.model].items():
        parts = []
        for n in rows:
            w = (torch.rand(n, K, device=dev, generator=g) * 2 - 1) * 0.05
            s = w.abs().amax(1, keepdim=True) / 448.0
            parts.append(Q.QuantPart.from_fp8((w / s).to(torch.float8_e4m3fn), s, dev))
            del w
        qw = Q.QuantWeight(parts)
        mb = sum(p.q.numel() for p in parts) / 1e6
        for M in a.m:
            x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
            S2 = Q.v2_splits(qw, M)
            ws2 = torch.empty(S2 * M * qw.N, dtype=torch.float32, device=dev)
            empty = torch.empty(0, dtype=torch.bfloat16, device=dev)
            t2 = Q._graph_time_us(lambda: Q._launch_v2(empty, ws2, x, qw, S2))
            S8 = Q.f8_decode_splits(qw, M)
            nsb = K // 256
            xq, xs = pgemm.act_quant(x)
            ops = torch.ops.hipserve
            rows = []
            for S in [S for S in range(1, nsb + 1) if nsb % S == 0 and nsb // S in Q.F8D_STEPS]:
                if -(-qw.N // 128) * S > 2048:
                    break
                ws8 = torch.empty(S * M * qw.N, dtype=torch.float32, device=dev)
                t8 = Q._graph_time_us(lambda: ops.fp8_decode_gemm(ws8, xq, xs, [p.q for p in parts],
                                                                  [p.rs for p in parts], S))
                rows.append(("fp8_w8a8" + ("*" if S == S8 else ""), S, t8))
            tq = Q._graph_time_us(lambda: ops.act_quant_fp8(xq, xs, x))
            for kern, S, t in [("v2_w8a16", S2, t2)] + rows + [("act_quant", 0, tq)]:
                print(json.dumps({"proj": name, "M": M, "kernel": kern, "splits": S, "us": round(t, 2),
                                  "weight_MB": round(mb, 2), "TBps": round(mb / t, 3) if S else None}), flush=True)


if __name__ == "__main__":
    main()
