"""Prefill GEMM units at prefill row counts: hipBLASLt (+ the separate GLU / residual-add
kernel) vs the packed-layout kernel (prefill_gemm_packed.hip: weights global -> VGPR; an
LDS-DMA form lost on every shape, profiles/r5_pgl_lds_dma_negative.log). Llama-3-8B / 70B layer shapes, random
operands, 4 weight copies streamed round-robin like a prefill step, interleaved rounds in
one process (cdna_hip_programming.md §5.4 rule 24): median and min per unit.

usage: python tools/bench_pgl.py [--m 8192] [--model 8b|70b|both] [--rounds 5]
"""
import argparse
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hipserve.ops import load_library  # noqa: E402

SHAPES = {
    "8b": [("plain", 6144, 4096), ("add", 4096, 4096), ("glu", 28672, 4096), ("add", 4096, 14336)],
    "70b": [("plain", 10240, 8192), ("add", 8192, 8192), ("glu", 57344, 8192), ("add", 8192, 28672)],
}


def _t(fn, n=4):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(n):
        fn(i)
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[8192])
    ap.add_argument("--model", default="8b")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    load_library()
    op = torch.ops.hipserve
    dev = torch.device("cuda", 0)
    models = ["8b", "70b"] if a.model == "both" else [a.model]
    for model in models:
        for M in a.m:
            for kind, N, K in SHAPES[model]:
                g = torch.Generator(device=dev).manual_seed(N + K)
                glu = kind == "glu"
                ncopy = 4 if N * K * 2 * 8 < (40 << 30) else 2
                ws = [((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
                      for _ in range(ncopy)]
                wps = []
                for w in ws:
                    wp = torch.empty(-(-N // 128) * 128 * K, device=dev, dtype=torch.bfloat16)
                    op.pack_decode_weight(wp, w, glu)
                    wps.append(wp)
                x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
                epi = 2 if glu else (1 if kind == "add" else 0)
                out = torch.empty(M, N // 2 if glu else N, device=dev, dtype=torch.bfloat16)
                res = torch.randn(M, N, device=dev).to(torch.bfloat16) if kind == "add" else None

                def blas(i):
                    y = F.linear(x, ws[i % ncopy])
                    if glu:
                        op.silu_and_mul(out, y)
                    elif res is not None:
                        res.add_(y)

                def packed(i):
                    op.prefill_gemm_packed(res if res is not None else out, x, wps[i % ncopy], N, epi, None, 1,
                                           1 << 30, 4)

                arms = {"blas": blas, "packed": packed}
                for f in arms.values():
                    f(0)
                torch.cuda.synchronize()
                ts = {k: [] for k in arms}
                for _ in range(a.rounds):
                    for k, f in arms.items():
                        ts[k].append(_t(f))
                flop = 2.0 * M * N * K
                row = {"model": model, "kind": kind, "M": M, "N": N, "K": K}
                for k, v in ts.items():
                    med = statistics.median(v)
                    row[k + "_ms"] = round(med, 4)
                    row[k + "_min_ms"] = round(min(v), 4)
                    row[k + "_pf"] = round(flop / med / 1e12, 3)
                print(row, flush=True)
                del ws, wps, x, out, res
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
