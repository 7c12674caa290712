#!/usr/bin/env python3
"""MoE prefill expert GEMMs, hipBLASLt's grouped GEMM (torch._grouped_mm: per-group
launches with a host read of the offsets on this ROCm build) vs the packed-layout grouped
kernel (prefill_gemm_packed.hip kGroup: one launch per GEMM, expert ids read on the
device), each with its own moe_align tile size and moe_gather, SiLU-GLU in between.

    python tools/bench_moe_prefill.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from hipserve.ops import gemm, load_library  # noqa: E402

DEV = "cuda"


def timed(fn, n=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b))
    return best


@torch.inference_mode()
def main():
    load_library()
    op = torch.ops.hipserve
    for name, E, H, I, k, T in [("qwen3-30b-a3b", 128, 2048, 768, 8, 8192), ("qwen3-30b-a3b", 128, 2048, 768, 8, 32768),
                                ("mixtral-8x7b", 8, 4096, 14336, 2, 8192)]:
        torch.manual_seed(0)
        w13 = (torch.randn(E, 2 * I, H, device=DEV) * 0.02).to(torch.bfloat16)
        w2 = (torch.randn(E, H, I, device=DEV) * 0.02).to(torch.bfloat16)
        p13 = torch.empty(E, 2 * I * H, dtype=torch.bfloat16, device=DEV)
        p2 = torch.empty(E, -(-H // 128) * 128 * I, dtype=torch.bfloat16, device=DEV)
        for e in range(E):
            op.pack_decode_weight(p13[e], w13[e], True)
            op.pack_decode_weight(p2[e], w2[e], False)
        x = torch.randn(T, H, device=DEV).to(torch.bfloat16)
        ids = torch.stack([torch.randperm(E, device=DEV)[:k] for _ in range(T)]).to(torch.int32)
        P = T * k
        flops = 2 * P * (2 * I * H + H * I)

        def route(tile, ids=ids):
            cap = -(-(P + E * (tile - 1)) // tile) * tile
            slots = torch.empty(cap, dtype=torch.int32, device=DEV)
            te = torch.empty(cap // tile, dtype=torch.int32, device=DEV)
            nt = torch.empty(1, dtype=torch.int32, device=DEV)
            ps = torch.empty(P, dtype=torch.int32, device=DEV)
            ends = torch.empty(E, dtype=torch.int32, device=DEV)
            op.moe_align(ids, E, tile, slots, te, nt, ps, ends)
            xs = torch.empty(cap, H, dtype=x.dtype, device=DEV)
            op.moe_gather(xs, x, slots, k)
            return cap, xs, te, nt, ends

        def blas():
            cap, xs, te, nt, ends = route(16)
            gu = torch._grouped_mm(xs, w13.transpose(1, 2), offs=ends)
            act = torch.empty(cap, I, dtype=x.dtype, device=DEV)
            op.silu_and_mul(act, gu)
            return torch._grouped_mm(act, w2.transpose(1, 2), offs=ends)

        ids0 = torch.zeros_like(ids)  # every pair on expert 0: the grouped kernel's own overhead

        def packed(ids=ids):
            tile = 128 * gemm.PW_WM
            cap, xs, te, nt, ends = route(tile, ids)
            act = torch.empty(cap, I, dtype=x.dtype, device=DEV)
            op.prefill_gemm_packed_grouped(act, xs, p13, 2 * I, 2, te, nt, gemm.PW_WM, gemm.PW_RW)
            y = torch.empty(cap, H, dtype=x.dtype, device=DEV)
            op.prefill_gemm_packed_grouped(y, act, p2, H, 0, te, nt, gemm.PW_WM, gemm.PW_RW)
            return y

        def dense():  # the same FLOPs as one dense packed GEMM pair on expert 0's weights
            tile = 128 * gemm.PW_WM
            cap, xs, te, nt, ends = route(tile)
            Pp = P // tile * tile
            act = torch.empty(Pp, I, dtype=x.dtype, device=DEV)
            op.prefill_gemm_packed(act, xs[:Pp], p13[0], 2 * I, 2, None, gemm.PW_WM, gemm.PW_GRID, gemm.PW_RW)
            y = torch.empty(Pp, H, dtype=x.dtype, device=DEV)
            op.prefill_gemm_packed(y, act, p2[0], H, 0, None, gemm.PW_WM, gemm.PW_GRID, gemm.PW_RW)
            return y

        def packed_gather():  # moe_gather fused into the first GEMM's X loads
            tile = 128 * gemm.PW_WM
            cap = -(-(P + E * (tile - 1)) // tile) * tile
            slots = torch.empty(cap, dtype=torch.int32, device=DEV)
            te = torch.empty(cap // tile, dtype=torch.int32, device=DEV)
            nt = torch.empty(1, dtype=torch.int32, device=DEV)
            ps = torch.empty(P, dtype=torch.int32, device=DEV)
            op.moe_align(ids, E, tile, slots, te, nt, ps)
            act = torch.empty(cap, I, dtype=x.dtype, device=DEV)
            op.prefill_gemm_packed_grouped(act, x, p13, 2 * I, 2, te, nt, gemm.PW_WM, gemm.PW_RW, slots, k)
            y = torch.empty(cap, H, dtype=x.dtype, device=DEV)
            op.prefill_gemm_packed_grouped(y, act, p2, H, 0, te, nt, gemm.PW_WM, gemm.PW_RW)
            return y

        tb, tp, td, t0 = timed(blas), timed(packed), timed(dense), timed(lambda: packed(ids0))
        tg = timed(packed_gather)
        print(json.dumps({"model": name, "tokens": T, "pairs": P, "grouped_mm_ms": round(tb, 3),
                          "packed_grouped_ms": round(tp, 3), "dense_packed_same_flops_ms": round(td, 3),
                          "packed_grouped_one_expert_ms": round(t0, 3),
                          "packed_gather_fused_ms": round(tg, 3), "grouped_mm_TFLOPs": round(flops / tb / 1e9, 1),
                          "packed_TFLOPs": round(flops / tp / 1e9, 1)}), flush=True)
        del w13, w2, p13, p2, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
