"""Prefill GEMM helpers: the FP8 W8A8 prefill (hipBLASLt's FP8 GEMM on the plain e4m3
weight, or the hand-written e4m3 kernel csrc/kernels/prefill_gemm.hip on the tiled
decode copy) and the start-up timing of the packed-layout bf16 prefill GEMM
(csrc/kernels/prefill_gemm_packed.hip) against hipBLASLt (``tune_packed``), which decides
whether a dense model keeps only its packed weight copy.

(Round 5 removed the bf16 / grouped families of prefill_gemm.hip: they lost to hipBLASLt
on every shipped config, VERDICT r4 "what's weak" 7.)
"""
from __future__ import annotations

import logging
import os

import torch
import torch.nn.functional as F

log = logging.getLogger("hipserve.pgemm")

# the kernels address each operand through 32-bit buffer offsets (prefill_gemm.hip
# pg_offsets_ok): larger operands go to hipBLASLt
OFFSET_LIMIT = 1 << 31


# ---- FP8 W8A8 prefill (the FP8-Dynamic checkpoints): per-token e4m3 activations x
# the e4m3 weights in the decode kernel's tiled layout, on the scaled FP8 MFMA
# (prefill_gemm.hip pgemm_f8_kernel). No bf16 shadow of the weights is needed.
FP8_MODE = os.environ.get("HIPSERVE_FP8_PREFILL", "1")
F8_MIN_ROWS = 128
# hipBLASLt's FP8 GEMM on a per-call re-laid-out copy (quant.f8_lib_weight, FP8_LIB
# "scratch") only above this many rows: the re-layout reads and writes the whole weight
# (~54 GB per Gemma-3-27B step), which a decode-only batch (graph buckets up to 512
# rows) cannot amortise — those run the hand-written kernel on the tiled copy
F8_SCRATCH_MIN_ROWS = 512


def f8_lib_ok(w, M: int) -> bool:
    """Route an M-row FP8 GEMM to hipBLASLt: a resident plain copy at any M % 16 == 0,
    the per-call scratch re-layout only for prefill-sized batches."""
    if M % 16:
        return False
    return getattr(w, "f8_plain", None) is not None or M > F8_SCRATCH_MIN_ROWS


def _f8_parts(w):
    from . import quant as Q
    if not isinstance(w, Q.QuantWeight) or not w.parts or not w.parts[0].q.is_cuda:
        return None
    if any(p.qtype != Q.FP8 or not p.tiled or p.K % 256 for p in w.parts) or len(w.parts) > 4:
        return None
    return w.parts


def f8_fits(w, glu: bool = False) -> bool:
    ps = _f8_parts(w)
    if ps is None or FP8_MODE == "0" or not hasattr(torch.ops.hipserve, "prefill_gemm_f8"):
        return False
    if glu:
        return len(ps) == 2 and ps[0].N == ps[1].N and ps[0].N % 128 == 0
    return all(p.N % 256 == 0 for p in ps)


def f8_use(w, M: int, glu: bool = False) -> bool:
    return (M >= F8_MIN_ROWS and f8_fits(w, glu) and M * w.parts[0].K < OFFSET_LIMIT
            and all(p.N * p.K < OFFSET_LIMIT for p in w.parts))


def act_quant(x: torch.Tensor):
    """Per-token dynamic e4m3: (xq uint8 [M, K], xs fp32 [M]) with x ~= e4m3(xq) * xs."""
    xq = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    xs = torch.empty(x.shape[0], dtype=torch.float32, device=x.device)
    torch.ops.hipserve.act_quant_fp8(xq, xs, x)
    return xq, xs


def f8_gemm(x: torch.Tensor, w, epi: int = 0, out: torch.Tensor | None = None, x8=None) -> torch.Tensor:
    """epi 0: out = x @ W^T (bf16 [M, N]); 1: out (the residual) += x @ W^T;
    2 / 3: W = (gate, up) parts, out = silu / gelu_tanh(x Wg^T) * (x Wu^T). ``x8``:
    x's per-token e4m3 copy already written by its producer (an RMSNorm with out8)."""
    ps = w.parts
    M = x.shape[0] if x is not None else x8[0].shape[0]
    dev = x.device if x is not None else x8[0].device
    out_given = out is not None
    if out is None:
        n = ps[0].N if epi in (2, 3) else w.N
        out = torch.empty(M, n, dtype=torch.bfloat16, device=dev)
    xq, xs = x8 if x8 is not None else act_quant(x)
    from . import quant as Q
    wp = Q.f8_lib_weight(w) if f8_lib_ok(w, M) else None
    if wp is not None:  # hipBLASLt FP8, row-wise scales, on the plain e4m3 weight
        y = torch._scaled_mm(xq.view(torch.float8_e4m3fn), wp.t(), scale_a=xs.reshape(-1, 1),
                             scale_b=w.f8_scale, out_dtype=torch.bfloat16)
        if epi == 0:
            if not out_given:
                return y
            out.copy_(y)
        elif epi == 1:
            out.add_(y)
        else:  # [gate | up] -> act
            (torch.ops.hipserve.silu_and_mul if epi == 2 else torch.ops.hipserve.gelu_and_mul)(out, y)
        return out
    torch.ops.hipserve.prefill_gemm_f8(out, xq, xs, [p.q for p in ps], [p.rs for p in ps], epi)
    return out


def f8_glu_q8(x: torch.Tensor, w, gelu: bool, x8=None):
    """FP8 gate|up on hipBLASLt FP8 (the plain e4m3 weight), then GLU and the per-token e4m3
    quantisation of act in one kernel (glu_quant): (xq, xs) of act for the FP8 down
    projection — no bf16 act round trip and no separate act_quant. None when the
    weight runs the hand-written kernel (the caller runs f8_gemm's GLU epilogue instead)."""
    from . import quant as Q
    M = x.shape[0]
    if getattr(w, "f8_scale", None) is None or not f8_lib_ok(w, M) or not hasattr(torch.ops.hipserve, "glu_quant"):
        return None
    wp = Q.f8_lib_weight(w)
    xq, xs = x8 if x8 is not None else act_quant(x)
    y = torch._scaled_mm(xq.view(torch.float8_e4m3fn), wp.t(), scale_a=xs.reshape(-1, 1),
                         scale_b=w.f8_scale, out_dtype=torch.bfloat16)
    inter = y.shape[1] // 2
    q8 = torch.empty(M, inter, dtype=torch.uint8, device=x.device)
    s8 = torch.empty(M, dtype=torch.float32, device=x.device)
    torch.ops.hipserve.glu_quant(None, q8, s8, y, gelu)
    return q8, s8


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
def tune_packed(units: list, M: int, device, ops) -> dict:
    """Start-up timing of the packed-layout prefill GEMM (prefill_gemm_packed.hip) against
    hipBLASLt on the layer's prefill units at M rows, random operands, 4 weight copies
    streamed like a prefill step: ``units`` = [(kind, N, K)] with kind "plain" (qkv),
    "add" (o / down: + residual add), "glu" (gate|up + SiLU-GLU). Returns the per-unit
    times and the layer totals; the runner keeps the single packed weight layout when
    the packed total is not slower."""
    from . import gemm as G

    op = torch.ops.hipserve
    rows, tp_, tb_ = [], 0.0, 0.0
    for kind, N, K in units:
        g = torch.Generator(device=device).manual_seed(N + K)
        ws = [((torch.rand(N, K, device=device, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(4)]
        wps = [G.PackedLinear(G.pack(w, glu=kind == "glu"), N, K, glu=kind == "glu") for w in ws]
        x = (torch.rand(M, K, device=device, generator=g) * 2 - 1).to(torch.bfloat16)
        if kind == "glu":
            act = torch.empty(M, N // 2, device=device, dtype=torch.bfloat16)
            t_b = _time(lambda i: ops.silu_and_mul(act, F.linear(x, ws[i])))
            t_p = _time(lambda i: G.packed_prefill(x, wps[i], 2, out=act))
        elif kind == "add":
            res = torch.randn(M, N, device=device).to(torch.bfloat16)
            t_b = _time(lambda i: res.add_(F.linear(x, ws[i])))
            t_p = _time(lambda i: G.packed_prefill(x, wps[i], 1, out=res))
        else:
            o = torch.empty(M, N, device=device, dtype=torch.bfloat16)
            t_b = _time(lambda i: F.linear(x, ws[i]))
            t_p = _time(lambda i: G.packed_prefill(x, wps[i], 0, out=o))
        rows.append({"kind": kind, "M": M, "N": N, "K": K, "blas_unit_ms": round(t_b, 4),
                     "packed_unit_ms": round(t_p, 4)})
        tp_, tb_ = tp_ + t_p, tb_ + t_b
        del ws, wps, x
    torch.cuda.empty_cache()
    r = {"units": rows, "packed_ms": round(tp_, 4), "blas_ms": round(tb_, 4)}
    log.info("packed prefill GEMM vs hipBLASLt: %s", r)
    return r
