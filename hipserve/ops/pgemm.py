"""Prefill GEMMs on the hand-written gfx950 kernel (csrc/kernels/prefill_gemm.hip) with
the layer's elementwise op fused into the tile store, chosen per projection shape by
timing it against hipBLASLt + the separate elementwise kernel at start-up:

* qkv        plain store                       (vs ``F.linear``)
* o / down   residual add in the epilogue      (vs ``F.linear`` + ``fused_add_rmsnorm``;
             the fused unit then runs a plain row RMSNorm)
* gate|up    SiLU-GLU in the epilogue          (vs ``F.linear`` + ``silu_and_mul``); each
             256-column tile streams 128 gate rows and the matching 128 up rows of
             the merged weight as stored (no repacked copy)
* MoE experts (``moe_grouped``, timed as a unit against hipBLASLt's grouped GEMM):
             one grouped launch per projection over the
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
# kernel schedule (prefill_gemm.hip): 1 = one-stage-ahead loop, 2 = half-tile pipeline (default;
# a one-barrier-per-K-tile schedule measured 11 % slower, profiles/r3_pgemm_pmc.md)
VARIANT = int(os.environ.get("HIPSERVE_PGEMM_VARIANT", "2"))
MIN_ROWS = 512        # below this hipBLASLt's smaller tiles win (and decode GEMMs take M <= 64)
CHOICE: dict[tuple, bool] = {}     # (kind, N, K) -> use prefill_gemm
REPORT: list[dict] = []


# the kernels address each operand through 32-bit buffer offsets (prefill_gemm.hip
# pg_offsets_ok): larger operands go to hipBLASLt
OFFSET_LIMIT = 1 << 31


def offsets_ok(M: int, K: int, N: int, elem: int = 2) -> bool:
    return M * K * elem < OFFSET_LIMIT and N * K * elem < OFFSET_LIMIT


def fits(w) -> bool:
    return isinstance(w, torch.Tensor) and w.is_cuda and w.dim() == 2 and w.dtype == torch.bfloat16 \
        and w.shape[0] % 256 == 0 and w.shape[1] % 64 == 0 and w.stride(1) == 1


def use(kind: str, w, M: int) -> bool:
    if MODE == "0" or M < MIN_ROWS or not fits(w) or not offsets_ok(M, w.shape[1], w.shape[0]):
        return False
    if MODE == "1":
        return True
    return CHOICE.get((kind, w.shape[0], w.shape[1]), False)


def gemm(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    out = torch.empty(x.shape[0], w.shape[0], device=x.device, dtype=x.dtype)
    torch.ops.hipserve.prefill_gemm(out, x, w, 0, VARIANT)
    return out


def gemm_add_(residual: torch.Tensor, x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """residual = bf16(bf16(x @ w.T) + residual), in place."""
    torch.ops.hipserve.prefill_gemm(residual, x, w, 1, VARIANT)
    return residual


def gemm_glu(x: torch.Tensor, w: torch.Tensor, gelu: bool = False) -> torch.Tensor:
    """act = silu(x @ Wg.T) * (x @ Wu.T) for the merged w = [Wg; Wu] (gelu: tanh-GELU,
    Gemma's GeGLU)."""
    act = torch.empty(x.shape[0], w.shape[0] // 2, device=x.device, dtype=x.dtype)
    torch.ops.hipserve.prefill_gemm(act, x, w, 3 if gelu else 2, VARIANT)
    return act


# ---- FP8 W8A8 prefill (the FP8-Dynamic checkpoints): per-token e4m3 activations x
# the e4m3 weights in the decode kernel's tiled layout, on the scaled FP8 MFMA
# (prefill_gemm.hip pgemm_f8_kernel). No bf16 shadow of the weights is needed.
FP8_MODE = os.environ.get("HIPSERVE_FP8_PREFILL", "1")
F8_MIN_ROWS = 128


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
    wp = Q.f8_lib_weight(w) if M % 16 == 0 else None
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
    if getattr(w, "f8_scale", None) is None or M % 16 or not hasattr(torch.ops.hipserve, "glu_quant"):
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


def moe_fits(w13, w2) -> bool:
    return (isinstance(w13, torch.Tensor) and w13.is_cuda and w13.dim() == 3
            and w13.dtype == torch.bfloat16 and w13.is_contiguous() and w2.is_contiguous()
            and w13.shape[1] % 256 == 0 and (w13.shape[1] // 2) % 128 == 0 and w13.shape[2] % 64 == 0
            and w2.shape[1] % 256 == 0 and w2.shape[2] % 64 == 0)


def moe_ok(w13, w2) -> bool:
    """Grouped expert GEMMs on the hand-written kernel (else hipBLASLt's grouped GEMM):
    ``1`` wherever the shapes fit, ``auto`` where the start-up timing chose it."""
    if MODE == "0" or not moe_fits(w13, w2):
        return False
    if MODE == "1":
        return True
    E, N13, H = w13.shape
    return any(CHOICE.get(("moe", E, N13 // 2, H, k), False) for k in range(1, 9))


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


def _tune_moe(E: int, inter: int, H: int, k: int, T: int, device, ops) -> dict:
    """The two grouped expert GEMMs of one MoE layer (+ SiLU-GLU) for T tokens routed
    uniformly at random: hand-written grouped kernel over moe_align's 256-row tiles vs
    hipBLASLt's grouped GEMM (torch._grouped_mm) over 16-row-padded groups."""
    op = torch.ops.hipserve
    g = torch.Generator(device=device).manual_seed(E + inter + H)
    w13 = ((torch.rand(E, 2 * inter, H, device=device, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
    w2 = ((torch.rand(E, H, inter, device=device, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
    x = (torch.rand(T, H, device=device, generator=g) * 2 - 1).to(torch.bfloat16)
    ids = torch.rand(T, E, device=device, generator=g).argsort(-1)[:, :k].int().contiguous()
    P = T * k

    def layout(tile):
        cap = -(-(P + E * (tile - 1)) // tile) * tile
        slots = torch.empty(cap, dtype=torch.int32, device=device)
        te = torch.empty(cap // tile, dtype=torch.int32, device=device)
        nt = torch.empty(1, dtype=torch.int32, device=device)
        ps = torch.empty(P, dtype=torch.int32, device=device)
        ends = torch.empty(E, dtype=torch.int32, device=device)
        op.moe_align(ids, E, tile, slots, te, nt, ps, ends)
        xs = torch.empty(cap, H, dtype=x.dtype, device=device)
        op.moe_gather(xs, x, slots, k)
        return cap, te, ends, xs

    cap, te, _, xs = layout(256)
    act = torch.empty(cap, inter, dtype=x.dtype, device=device)
    y = torch.empty(cap, H, dtype=x.dtype, device=device)

    def p_moe(i):
        op.prefill_gemm_grouped(act, xs, w13, te, 2, VARIANT)
        op.prefill_gemm_grouped(y, act, w2, te, 0, VARIANT)

    t_p = _time(p_moe, reps=2)
    cap16, _, ends, xs16 = layout(16)
    act16 = torch.empty(cap16, inter, dtype=x.dtype, device=device)

    def b_moe(i):
        ops.silu_and_mul(act16, torch._grouped_mm(xs16, w13.transpose(1, 2), offs=ends))
        torch._grouped_mm(act16, w2.transpose(1, 2), offs=ends)

    t_b = _time(b_moe, reps=2)
    key = ("moe", E, inter, H, k)
    CHOICE[key] = t_p < t_b * 0.99
    r = {"kind": "moe", "M": T, "E": E, "I": inter, "H": H, "top_k": k, "blas_unit_ms": round(t_b, 4),
         "pgemm_unit_ms": round(t_p, 4), "pgemm": CHOICE[key]}
    log.info("prefill GEMM %s", r)
    return r


@torch.inference_mode()
def tune(units: dict, M: int, device, ops) -> list[dict]:
    """units: {(kind, N, K)} with kind in {"plain", "add", "glu"} and
    ("moe", E, I, H, top_k); times both ways (dense kinds on 4 weight copies, streaming
    weights like a prefill step) and fills CHOICE."""
    if MODE == "0":
        return []
    out = []
    for u in sorted(units):
        if u[0] == "moe":
            out.append(_tune_moe(*u[1:], M, device, ops))
            continue
        kind, N, K = u
        if N % 256 or K % 64:
            continue
        g = torch.Generator(device=device).manual_seed(N + K)
        ws = [((torch.rand(N, K, device=device, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(4)]
        x = ((torch.rand(M, K, device=device, generator=g) * 2 - 1)).to(torch.bfloat16)
        if kind == "glu":
            act = torch.empty(M, N // 2, device=device, dtype=torch.bfloat16)
            t_b = _time(lambda i: ops.silu_and_mul(act, F.linear(x, ws[i])))
            t_p = _time(lambda i: torch.ops.hipserve.prefill_gemm(act, x, ws[i], 2, VARIANT))
        elif kind == "add":
            res = torch.randn(M, N, device=device).to(torch.bfloat16)
            nw = torch.ones(N, device=device, dtype=torch.bfloat16)
            xn = torch.empty_like(res)
            t_b = _time(lambda i: ops.fused_add_rmsnorm(xn, F.linear(x, ws[i]), res, nw, 1e-5))

            def p_add(i):
                torch.ops.hipserve.prefill_gemm(res, x, ws[i], 1, VARIANT)
                ops.rmsnorm(xn, res, nw, 1e-5)
            t_p = _time(p_add)
        else:
            o = torch.empty(M, N, device=device, dtype=torch.bfloat16)
            t_b = _time(lambda i: F.linear(x, ws[i]))
            t_p = _time(lambda i: torch.ops.hipserve.prefill_gemm(o, x, ws[i], 0, VARIANT))
        CHOICE[(kind, N, K)] = t_p < t_b * 0.99
        r = {"kind": kind, "M": M, "N": N, "K": K, "blas_unit_ms": round(t_b, 4), "pgemm_unit_ms": round(t_p, 4),
             "pgemm": CHOICE[(kind, N, K)]}
        out.append(r)
        log.info("prefill GEMM %s", r)
        del ws, x
    torch.cuda.empty_cache()
    REPORT.extend(out)
    return out


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
