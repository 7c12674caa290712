"""Prefill GEMMs on the hand-written gfx950 kernel (csrc/kernels/prefill_gemm.hip) with
the layer's elementwise op fused into the tile store, chosen per projection shape by
timing it against hipBLASLt + the separate elementwise kernel at start-up:

* qkv        plain store                       (vs ``F.linear``)
* o / down   residual add in the epilogue      (vs ``F.linear`` + ``fused_add_rmsnorm``;
             the fused unit then runs a plain row RMSNorm)
* gate|up    SiLU-GLU in the epilogue          (vs ``F.linear`` + ``silu_and_mul``); each
             256-column tile streams 128 gate rows and the matching 128 up rows of
             the merged weight as stored (no repacked copy)
* MoE experts (``grouped_moe``): one grouped launch per projection over the
             expert-sorted 256-row tiles of ``moe_align`` (device-side expert ids —
             no host round trip, unlike ``torch._grouped_mm`` on this ROCm build),
             SiLU-GLU in the gate|up epilogue

``HIPSERVE_PREFILL_GEMM``: ``auto`` (default: the timed choice), ``1`` (always, where
the shape fits), ``0`` (hipBLASLt only).
"""
from __future__ import annotations

import logging
import os

import torch
import torch.nn.functional as F

log = logging.getLogger("hipserve.pgemm")

MODE = os.environ.get("HIPSERVE_PREFILL_GEMM", "auto")
MIN_ROWS = 512        # below this hipBLASLt's smaller tiles win (and decode GEMMs take M <= 64)
CHOICE: dict[tuple, bool] = {}     # (kind, N, K) -> use prefill_gemm
REPORT: list[dict] = []


def fits(w) -> bool:
    return isinstance(w, torch.Tensor) and w.is_cuda and w.dim() == 2 and w.dtype == torch.bfloat16 \
        and w.shape[0] % 256 == 0 and w.shape[1] % 64 == 0 and w.stride(1) == 1


def use(kind: str, w, M: int) -> bool:
    if MODE == "0" or M < MIN_ROWS or not fits(w):
        return False
    if MODE == "1":
        return True
    return CHOICE.get((kind, w.shape[0], w.shape[1]), False)


def gemm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    out = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=x.dtype)
    torch.ops.hipserve.prefill_gemm(out, x, w, 0)
    return out


def gemm_add_(residual: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """residual = bf16(bf16(x @ w.T) + residual), in place."""
    torch.ops.hipserve.prefill_gemm(residual, x, w, 1)
    return residual


def gemm_glu(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """act = silu(x @ Wg.T) * (x @ Wu.T) for the merged w = [Wg; Wu]."""
    act = torch.empty(x.shape[0], w.shape[0] // 2, device=x.device, dtype=x.dtype)
    torch.ops.hipserve.prefill_gemm(act, x, w, 2)
    return act


def moe_ok(w13, w2) -> bool:
    return (MODE != "0" and isinstance(w13, torch.Tensor) and w13.is_cuda and w13.dim() == 3
            and w13.dtype == torch.bfloat16 and w13.is_contiguous() and w2.is_contiguous()
            and w13.shape[1] % 256 == 0 and (w13.shape[1] // 2) % 128 == 0 and w13.shape[2] % 64 == 0
            and w2.shape[1] % 256 == 0 and w2.shape[2] % 64 == 0)


def _time(fn, reps=3):
    fn(0)
    torch.cuda.synchronize()
    best = float("inf")
    for r in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(4):
            fn(i)
        b.record()
        b.synchronize()
        best = min(best, a.elapsed_time(b) / 4)
    return best


@torch.inference_mode()
def tune(units: dict, M: int, device, ops) -> list[dict]:
    """units: {(kind, N, K)} with kind in {"plain", "add", "glu"}; times both ways on
    4 weight copies (streams weights like a prefill step) and fills CHOICE."""
    if MODE == "0":
        return []
    out = []
    for (kind, N, K) in sorted(units):
        if N % 256 or K % 64:
            continue
        g = torch.Generator(device=device).manual_seed(N + K)
        ws = [((torch.rand(N, K, device=device, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(4)]
        x = ((torch.rand(M, K, device=device, generator=g) * 2 - 1)).to(torch.bfloat16)
        if kind == "glu":
            act = torch.empty(M, N // 2, device=device, dtype=torch.bfloat16)
            t_b = _time(lambda i: ops.silu_and_mul(act, F.linear(x, ws[i])))
            t_p = _time(lambda i: torch.ops.hipserve.prefill_gemm(act, x, ws[i], 2))
        elif kind == "add":
            res = torch.randn(M, N, device=device).to(torch.bfloat16)
            nw = torch.ones(N, device=device, dtype=torch.bfloat16)
            xn = torch.empty_like(res)
            t_b = _time(lambda i: ops.fused_add_rmsnorm(xn, F.linear(x, ws[i]), res, nw, 1e-5))

            def p_add(i):
                torch.ops.hipserve.prefill_gemm(res, x, ws[i], 1)
                ops.rmsnorm(xn, res, nw, 1e-5)
            t_p = _time(p_add)
        else:
            o = torch.empty(M, N, device=device, dtype=torch.bfloat16)
            t_b = _time(lambda i: F.linear(x, ws[i]))
            t_p = _time(lambda i: torch.ops.hipserve.prefill_gemm(o, x, ws[i], 0))
        CHOICE[(kind, N, K)] = t_p < t_b * 0.99
        r = {"kind": kind, "M": M, "N": N, "K": K, "blas_unit_ms": round(t_b, 4), "pgemm_unit_ms": round(t_p, 4),
             "pgemm": CHOICE[(kind, N, K)]}
        out.append(r)
        log.info("prefill GEMM %s", r)
        del ws, x
    torch.cuda.empty_cache()
    REPORT.extend(out)
    return out
