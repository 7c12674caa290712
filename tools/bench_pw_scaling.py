#!/usr/bin/env python3
"""Packed-layout prefill GEMM (prefill_gemm_packed.hip) time vs K at fixed M x N, against
hipBLASLt: the slope is the main loop's cost per 64-deep K stage, the intercept the
per-tile prologue + epilogue that a workgroup does not overlap with MFMA work. (The
diagnostic no-weight-load / no-X-staging variants behind profiles/r4_pw_scaling_v3.log
were removed from the kernel library in round 5.)
usage: python tools/bench_pw_scaling.py [--m 8192] [--n 28672]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from hipserve.ops import load_library


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--n", type=int, default=28672)
    ap.add_argument("--ks", default="1024,2048,4096,8192")
    ap.add_argument("--epi", type=int, default=0)
    a = ap.parse_args()
    load_library()
    op = torch.ops.hipserve
    M, N = a.m, a.n
    for K in (int(k) for k in a.ks.split(",")):
        x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
        ws = [((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(4)]
        wps = []
        for w in ws:
            wp = torch.empty(-(-N // 128) * 128 * K, device="cuda", dtype=torch.bfloat16)
            op.pack_decode_weight(wp, w, a.epi in (2, 3))
            wps.append(wp)
        out = torch.empty(M, N // 2 if a.epi in (2, 3) else N, device="cuda", dtype=torch.bfloat16)

        def t(fn):
            fn()
            torch.cuda.synchronize()
            best = 1e9
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                best = min(best, e0.elapsed_time(e1) / 4)
            return best
        r = {"M": M, "N": N, "K": K, "epi": a.epi, "blas_ms": round(t(lambda: [F.linear(x, w) for w in ws]), 4)}
        for wm in (1, 2):
            for rw in ((4,) if wm == 1 else (2,)):
                r[f"wm{wm}_rw{rw}_ms"] = round(t(lambda: [op.prefill_gemm_packed(out, x, wp, N, a.epi, None, wm, 0, rw)
                                                          for wp in wps]), 4)
        # one tile per workgroup (non-persistent launch)
        for rw in (4, 5):
            r[f"wm1_rw{rw}_1tile_ms"] = round(t(lambda: [op.prefill_gemm_packed(out, x, wp, N, a.epi, None, 1, 1 << 30, rw)
                                                         for wp in wps]), 4)
        r["wm1_ms"] = min(v for k, v in r.items() if k.startswith("wm1_"))
        r["wm1_TFs"] = round(2 * M * N * K / r["wm1_ms"] / 1e9, 1)
        r["blas_TFs"] = round(2 * M * N * K / r["blas_ms"] / 1e9, 1)
        print(json.dumps(r), flush=True)
        del x, ws, wps, out
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
