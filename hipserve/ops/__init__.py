"""hipserve op library.

``KernelOps`` calls the hand-written gfx950 kernels in ``hipserve/_C.so``
(``torch.ops.hipserve.*``). ``ReferenceOps`` is the plain-PyTorch oracle used by
the CPU plumbing engine and by the numerics tests. The choice is made ONCE, when
an engine is built for a device — never per call. On a GPU device the native
library is mandatory: a missing/unloadable ``_C.so`` raises instead of silently
falling back to PyTorch.
"""
from __future__ import annotations

import os
import threading

import torch

from . import reference as ref

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
_lock = threading.Lock()
_loaded = False


def library_path() -> str:
    return _LIB


def load_library(build_if_missing: bool = False) -> str:
    """Load hipserve/_C.so into torch.ops (idempotent). Raises if unavailable."""
    global _loaded
    with _lock:
        if _loaded:
            return _LIB
        if not os.path.exists(_LIB) and build_if_missing:
            from .._build import build_kernels

            build_kernels()
        if not os.path.exists(_LIB):
            raise RuntimeError(
                f"hipserve native kernels not built ({_LIB} missing): run `python -m hipserve._build`")
        torch.ops.load_library(_LIB)
        _loaded = True
        return _LIB


def native_available() -> bool:
    try:
        load_library()
        return True
    except Exception:
        return False


class KernelOps:
    """gfx950 HIP kernels (all outputs written in place; graph-capturable)."""

    name = "hip"

    def __init__(self):
        load_library()
        self._op = torch.ops.hipserve

    def rmsnorm(self, out, x, w, eps, out8=None):
        """out8: (e4m3 [rows, hidden] uint8, scales fp32 [rows]) per-token FP8 copy of out."""
        self._op.rmsnorm(out, x, w, eps, *(out8 if out8 is not None else (None, None)))
        return out

    def fused_add_rmsnorm(self, out, x, residual, w, eps, out8=None):
        self._op.fused_add_rmsnorm(out, x, residual, w, eps, *(out8 if out8 is not None else (None, None)))
        return out

    def silu_and_mul(self, out, x):
        self._op.silu_and_mul(out, x)
        return out

    def gelu_and_mul(self, out, x):
        self._op.gelu_and_mul(out, x)
        return out

    def qk_rmsnorm(self, qkv, q_w, k_w, nq, nkv, D, eps):
        self._op.qk_rmsnorm(qkv, q_w, k_w, nq, nkv, D, eps)

    def fill_uniform(self, out, row0, col0, gcols, key, scale):
        self._op.fill_uniform(out, row0, col0, gcols, key, scale)
        return out

    def rope_cache(self, qkv, positions, slots, cos_sin, k_cache, v_cache, nq, nkv, D, mode):
        self._op.rope_cache(qkv, positions, slots, cos_sin, k_cache, v_cache, nq, nkv, D, mode)

    def paged_decode(self, out, q, k_cache, v_cache, block_tables, context_lens, tmp_out, tmp_ml,
                     nq, nkv, part_size, scale, window=0, out16=None):
        self._op.paged_decode(out, q, k_cache, v_cache, block_tables, context_lens, tmp_out, tmp_ml,
                              nq, nkv, part_size, scale, window, out16)
        return out

    def prefill_attention(self, out, q, k_cache, v_cache, block_tables, cu_q, ctx_lens, tiles,
                          nq, nkv, scale, window=0):
        self._op.prefill_attention(out, q, k_cache, v_cache, block_tables, cu_q, ctx_lens, tiles,
                                   nq, nkv, scale, window)
        return out

    def sample(self, out_tok, out_lp, logits, temperature, top_k, top_p, seeds, steps, two_rounds=True):
        """two_rounds=False: no row combines top-k with top-p (the multi-CU sampler's
        second fine-histogram round is then a no-op and is not launched)."""
        self._op.sample(out_tok, out_lp, logits, temperature, top_k, top_p, seeds, steps, two_rounds)

    def penalty_apply(self, logits, slot, pres, freq, rep, counts, seen):
        self._op.penalty_apply(logits, slot, pres, freq, rep, counts, seen)

    def penalty_update(self, tok, slot, counts, seen):
        self._op.penalty_update(tok, slot, counts, seen)

    def penalty_init(self, counts, seen, slots, off, n_prompt, toks):
        self._op.penalty_init(counts, seen, slots, off, n_prompt, toks)

    def top_logprobs(self, logits, nreq, out_ids, out_lp):
        self._op.top_logprobs(logits, nreq, out_ids, out_lp)

    # ---- vision tower (csrc/kernels/vision.hip)
    def layernorm(self, out, x, w, b, eps, residual=None):
        self._op.layernorm(out, x, w, b, residual, eps)
        return out

    def gelu_(self, x, tanh):
        self._op.gelu_(x, tanh)
        return x

    VISION_TILE = 128  # query rows per attention workgroup (4 waves x 32)

    def vision_meta(self, geo, nh, D):
        """(cu_seqlens, tiles) device tensors of an image batch for vision_attention."""
        import numpy as np

        cu = geo.cu_seqlens
        tiles = np.array([(s, r) for s in range(len(cu) - 1) for r in range(0, int(cu[s + 1] - cu[s]),
                                                                          self.VISION_TILE)], np.int32)
        dev = torch.device("cuda", torch.cuda.current_device())
        return (torch.from_numpy(cu.astype(np.int32)).to(dev), torch.from_numpy(tiles.reshape(-1, 2)).to(dev))

    def vision_attention(self, out, qkv, cos_sin, cu_seqlens, nh, D, scale, meta=None):
        cu, tiles = meta
        self._op.vision_attention(out, qkv, cos_sin, cu, tiles, nh, D, scale)
        return out


class ReferenceOps:
    """PyTorch reference path (CPU plumbing engine / numerics oracle)."""

    name = "reference"

    def fill_uniform(self, out, row0, col0, gcols, key, scale):
        return ref.fill_uniform(out, row0, col0, gcols, key, scale)

    def rmsnorm(self, out, x, w, eps, out8=None):
        assert out8 is None, "the FP8 copy is a HIP-kernel output"
        out.copy_(ref.rmsnorm(x, w, eps))
        return out

    def fused_add_rmsnorm(self, out, x, residual, w, eps, out8=None):
        assert out8 is None, "the FP8 copy is a HIP-kernel output"
        y, r = ref.fused_add_rmsnorm(x, residual, w, eps)
        residual.copy_(r)
        out.copy_(y)
        return out

    def silu_and_mul(self, out, x):
        out.copy_(ref.silu_and_mul(x))
        return out

    def gelu_and_mul(self, out, x):
        out.copy_(ref.gelu_and_mul(x))
        return out

    def qk_rmsnorm(self, qkv, q_w, k_w, nq, nkv, D, eps):
        ref.qk_rmsnorm(qkv, q_w, k_w, nq, nkv, D, eps)

    def rope_cache(self, qkv, positions, slots, cos_sin, k_cache, v_cache, nq, nkv, D, mode):
        ref.rope_cache(qkv, positions, slots, cos_sin, k_cache, v_cache, nq, nkv, D, mode)

    def paged_decode(self, out, q, k_cache, v_cache, block_tables, context_lens, tmp_out, tmp_ml,
                     nq, nkv, part_size, scale, window=0, out16=None):
        B = context_lens.shape[0]
        D = k_cache.shape[3]
        out[:B, : nq * D].copy_(ref.paged_decode(q, k_cache, v_cache, block_tables, context_lens,
                                                 nq, nkv, scale, window).view(B, nq * D))
        return out

    def prefill_attention(self, out, q, k_cache, v_cache, block_tables, cu_q, ctx_lens, tiles,
                          nq, nkv, scale, window=0):
        D = k_cache.shape[3]
        T = int(cu_q[-1])
        out[:T, : nq * D].copy_(ref.prefill_attention(q, k_cache, v_cache, block_tables, cu_q,
                                                      ctx_lens, nq, nkv, scale, window).view(T, nq * D))
        return out

    def penalty_apply(self, logits, slot, pres, freq, rep, counts, seen):
        ref.penalty_apply(logits, slot, pres, freq, rep, counts, seen)

    def penalty_update(self, tok, slot, counts, seen):
        ref.penalty_update(tok, slot, counts, seen)

    def penalty_init(self, counts, seen, slots, off, n_prompt, toks):
        ref.penalty_init(counts, seen, slots, off, n_prompt, toks)

    def top_logprobs(self, logits, nreq, out_ids, out_lp):
        ref.top_logprobs(logits, nreq, out_ids, out_lp)

    # ---- vision tower (Qwen3-VL ViT)
    def layernorm(self, out, x, w, b, eps, residual=None):
        if residual is None:
            out.copy_(ref.layernorm(x, w, b, eps))
        else:
            y, r = ref.add_layernorm(x, residual, w, b, eps)
            residual.copy_(r)
            out.copy_(y)
        return out

    def gelu_(self, x, tanh):
        x.copy_(ref.gelu(x, tanh))
        return x

    def vision_attention(self, out, qkv, cos_sin, cu_seqlens, nh, D, scale, meta=None):
        ref.vision_rope(qkv, cos_sin, nh, D)
        out.copy_(ref.vision_attention(qkv, cu_seqlens, nh, D, scale))
        return out

    def sample(self, out_tok, out_lp, logits, temperature, top_k, top_p, seeds, steps, two_rounds=True):
        t, lp = ref.sample(logits, temperature, top_k, top_p, seeds, steps, bf16_row=False)
        n = t.shape[0]
        out_tok[:n].copy_(t)
        if out_lp.numel():
            out_lp[:n].copy_(lp)


def get_ops(device: torch.device | str):
    device = torch.device(device)
    if device.type == "cuda":
        return KernelOps()
    return ReferenceOps()
