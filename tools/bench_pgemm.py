#!/usr/bin/env python3
"""The hand-written prefill GEMMs (packed bf16: prefill_gemm_packed.hip; FP8 W8A8:
prefill_gemm.hip) vs hipBLASLt
(``F.linear``) on the Llama-3-8B / 70B-TP8 prefill shapes at M = 8192 rows, random
[-1, 1) operands (cdna_hip_programming.md rule 25), one weight per layer so the 32
calls stream 32 different weights. Also the fused units: GLU (gate|up GEMM + SiLU·mul)
and residual add (o / down GEMM + add) vs hipBLASLt + the separate elementwise
kernel. One JSON line per shape plus a markdown table.

usage: python tools/bench_pgemm.py [--m 8192] [--layers 8] [--model 8b|70b-tp8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=8192)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--model", default="8b")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--fp8", action="store_true", help="also the FP8 W8A8 kernel (act quant + e4m3 MFMA GEMM)")
    a = ap.parse_args()
    from hipserve.ops import KernelOps

    ops = KernelOps()
    op = torch.ops.hipserve
    dev = "cuda"
    H, I, NQKV, HO = {"8b": (4096, 14336, 6144, 4096), "70b-tp8": (8192, 3584, 1280, 1024),
                      "gemma27b": (5376, 21504, 8192, 4096)}[a.model]
    shapes = {"qkv": (NQKV, H), "o": (H, HO), "gu": (2 * I, H), "down": (H, I)}
    M, L = a.m, a.layers

    def rnd(*s):
        return (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)

    def time_fn(fn):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        return best / L

    rows = []
    for name, (N, K) in shapes.items():
        x = rnd(M, K)
        ws = [rnd(N, K) * 0.05 for _ in range(L)]
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        t_blas = time_fn(lambda: [F.linear(x, w) for w in ws])
        # the packed-layout kernel (prefill_gemm_packed.hip) on the decode copy of each weight
        glu_pack = name == "gu"
        wps = []
        for w in ws:
            wp = torch.empty(-(-N // 128) * 128 * K, device=dev, dtype=torch.bfloat16)
            op.pack_decode_weight(wp, w, False)
            wps.append(wp)
        t_pw = {wm: time_fn(lambda: [op.prefill_gemm_packed(out, x, wp, N, 0, None, wm) for wp in wps]) for wm in (1, 2)}
        r = {"shape": name, "M": M, "N": N, "K": K, "blas_ms": round(t_blas, 4),
             "packed_wm1_ms": round(t_pw[1], 4), "packed_wm2_ms": round(t_pw[2], 4),
             "blas_TFs": round(2 * M * N * K / t_blas / 1e9, 1),
             "packed_TFs": round(2 * M * N * K / min(t_pw.values()) / 1e9, 1)}
        if a.fp8:
            from hipserve.ops import pgemm, quant as Q

            qws = []
            for w in ws:
                sc = w.float().abs().amax(1, keepdim=True) / 448.0
                qws.append(Q.QuantWeight([Q.QuantPart.from_fp8((w.float() / sc).to(torch.float8_e4m3fn), sc, dev)]))
            t_q = time_fn(lambda: [pgemm.act_quant(x) for _ in qws])
            t_f8 = time_fn(lambda: [pgemm.f8_gemm(x, q, 0, out) for q in qws])
            r.update({"fp8_ms": round(t_f8, 4), "fp8_quant_ms": round(t_q, 4),
                      "fp8_TFs": round(2 * M * N * K / t_f8 / 1e9, 1)})
            del qws
            # hipBLASLt FP8 with row-wise scales (torch._scaled_mm) on a plain [N, K] e4m3
            # copy, for reference: the library's FP8 rate on the same shapes
            try:
                w8 = [(w.float() / (w.float().abs().amax(1, keepdim=True) / 448.0)).to(torch.float8_e4m3fn)
                      for w in ws]
                sw = [(w.float().abs().amax(1) / 448.0).reshape(1, -1).contiguous() for w in ws]
                xq8, xs8 = pgemm.act_quant(x)
                xf8 = xq8.view(torch.float8_e4m3fn)
                sx = xs8.reshape(-1, 1).contiguous()
                t_sm = time_fn(lambda: [torch._scaled_mm(xf8, w.t(), scale_a=sx, scale_b=s_, out_dtype=torch.bfloat16)
                                        for w, s_ in zip(w8, sw)])
                r.update({"blas_fp8_rowwise_ms": round(t_sm, 4), "blas_fp8_TFs": round(2 * M * N * K / t_sm / 1e9, 1)})
                del w8
            except Exception as e:  # noqa: BLE001 - report what the library refused
                r["blas_fp8_rowwise"] = f"unsupported: {type(e).__name__}: {str(e)[:120]}"
        if name == "gu":  # GEMM + SiLU-GLU unit
            act = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)

            def blas_glu():
                for w in ws:
                    ops.silu_and_mul(act, F.linear(x, w))
            r["blas_unit_ms"] = round(time_fn(blas_glu), 4)
            for w, wp in zip(ws, wps):
                op.pack_decode_weight(wp, w, True)
            r["packed_unit_ms"] = {wm: round(time_fn(lambda: [op.prefill_gemm_packed(act, x, wp, N, 2, None, wm)
                                                              for wp in wps]), 4) for wm in (1, 2)}
        if name in ("o", "down"):  # GEMM + residual add unit
            res = rnd(M, N)

            def blas_add():
                for w in ws:
                    res.add_(F.linear(x, w))
            r["blas_unit_ms"] = round(time_fn(blas_add), 4)
            r["packed_unit_ms"] = {wm: round(time_fn(lambda: [op.prefill_gemm_packed(res, x, wp, N, 1, None, wm)
                                                              for wp in wps]), 4) for wm in (1, 2)}
        rows.append(r)
        print(json.dumps(r), flush=True)
        del ws, wps, x, out
        torch.cuda.empty_cache()
    print(f"\n| shape | M x N x K | hipBLASLt ms (TF/s) | packed wm1 / wm2 ms (TF/s) "
          f"| unit: hipBLASLt + ew | unit: packed | FP8 quant + GEMM ms (TF/s) |")
    print("|---|---|---:|---:|---:|---:|---:|")
    for r in rows:
        f8 = f"{r['fp8_ms']} ({r['fp8_TFs']})" if "fp8_ms" in r else "—"
        print(f"| {r['shape']} | {r['M']}x{r['N']}x{r['K']} | {r['blas_ms']} ({r['blas_TFs']}) | "
              f"{r['packed_wm1_ms']} / {r['packed_wm2_ms']} ({r['packed_TFs']}) | "
              f"{r.get('blas_unit_ms', '—')} | {r.get('packed_unit_ms', '—')} | {f8} |")


if __name__ == "__main__":
    main()
