"""Plain-PyTorch fp32 reference implementations of every hipserve kernel.

These are the numerics oracles for the gfx950 kernels (tests compare the HIP op
against these) and the compute path of the CPU plumbing engine (tests/CI without
a GPU). They use exactly the same tensor layouts as the kernels:

* ``k_cache [num_blocks, nkv, block_size, D]``
* ``v_cache [num_blocks, nkv, D, block_size]`` (transposed per block)
* ``cos_sin [max_pos, D]`` = ``[cos(D/2) | sin(D/2)]`` fp32
"""
from __future__ import annotations

import math

import numpy as np
import torch


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * inv * w.float()).to(x.dtype)


def fused_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """Returns (normed, new_residual); residual is rounded to x.dtype first."""
    r = (x.float() + residual.float()).to(x.dtype)
    return rmsnorm(r, w, eps), r


def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    inter = x.shape[-1] // 2
    g, u = x[..., :inter].float(), x[..., inter:].float()
    return (torch.nn.functional.silu(g) * u).to(x.dtype)


def gelu_and_mul(x: torch.Tensor) -> torch.Tensor:
    """tanh-GELU(gate) * up (Gemma GeGLU, HF gelu_pytorch_tanh)."""
    inter = x.shape[-1] // 2
    g, u = x[..., :inter].float(), x[..., inter:].float()
    return (torch.nn.functional.gelu(g, approximate="tanh") * u).to(x.dtype)


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    """LayerNorm over the last dim (fp32 statistics, x.dtype out)."""
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def add_layernorm(x: torch.Tensor, residual: torch.Tensor, w, b, eps: float):
    """(LayerNorm(r), r) with r = residual + x rounded to x.dtype first."""
    r = (x.float() + residual.float()).to(x.dtype)
    return layernorm(r, w, b, eps), r


def gelu(x: torch.Tensor, tanh: bool) -> torch.Tensor:
    return torch.nn.functional.gelu(x.float(), approximate="tanh" if tanh else "none").to(x.dtype)


def vision_rope(qkv: torch.Tensor, cos_sin: torch.Tensor, nh: int, D: int):
    """In place: rotate-half RoPE of the q and k heads of a ViT qkv [T, 3*nh*D] with one
    fp32 table row per token ([cos(D/2) | sin(D/2)], the 2D row/column angles)."""
    T = qkv.shape[0]
    half = D // 2
    c, s = cos_sin[:T, None, :half].float(), cos_sin[:T, None, half:].float()
    for j in range(2):
        x = qkv[:, j * nh * D:(j + 1) * nh * D].view(T, nh, D)
        a, b = x[..., :half].float(), x[..., half:].float()
        x.copy_(torch.cat([a * c - b * s, b * c + a * s], -1).to(x.dtype))


def vision_attention(qkv: torch.Tensor, cu_seqlens, nh: int, D: int, scale: float) -> torch.Tensor:
    """Bidirectional attention within each segment [cu[i], cu[i+1]) of a ViT qkv
    [T, 3*nh*D] (fp32 math) -> [T, nh*D]."""
    T = qkv.shape[0]
    q = qkv[:, : nh * D].view(T, nh, D).float()
    k = qkv[:, nh * D:2 * nh * D].view(T, nh, D).float()
    v = qkv[:, 2 * nh * D:].view(T, nh, D).float()
    out = torch.empty(T, nh, D, dtype=torch.float32, device=qkv.device)
    cu = [int(x) for x in cu_seqlens]
    for a, b in zip(cu[:-1], cu[1:]):
        s = torch.einsum("qhd,khd->hqk", q[a:b], k[a:b]) * scale
        out[a:b] = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), v[a:b])
    return out.view(T, nh * D).to(qkv.dtype)


def qk_rmsnorm(qkv: torch.Tensor, q_w: torch.Tensor, k_w: torch.Tensor, nq: int, nkv: int, D: int, eps: float):
    """In place: RMSNorm over head_dim of every q head (weight q_w) and k head (k_w)."""
    T = qkv.shape[0]
    if T == 0:
        return
    q = qkv[:, : nq * D].view(T, nq, D)
    k = qkv[:, nq * D:(nq + nkv) * D].view(T, nkv, D)
    q.copy_(rmsnorm(q, q_w, eps))
    k.copy_(rmsnorm(k, k_w, eps))


def rope_cos_sin(head_dim: int, max_pos: int, theta: float, scaling: dict | None = None,
                 rotary_dim: int | None = None) -> torch.Tensor:
    """fp32 [max_pos, D] table = [cos | sin] with optional Llama-3 frequency scaling."""
    rd = rotary_dim or head_dim
    inv_freq = 1.0 / (theta ** (torch.arange(0, rd, 2, dtype=torch.float64) / rd))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv_freq
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv_freq / factor, inv_freq)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv_freq / factor + smooth * inv_freq, scaled)
        inv_freq = scaled
    elif scaling and scaling.get("rope_type", scaling.get("type")) == "linear":
        inv_freq = inv_freq / scaling["factor"]
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv_freq)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().contiguous()


def apply_rope(x: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor, mode: int) -> torch.Tensor:
    """x [T, H, D] -> rotated (fp32 math, x.dtype out)."""
    D = x.shape[-1]
    half = D // 2
    cs = cos_sin[pos.long()]  # [T, D]
    c, s = cs[:, None, :half], cs[:, None, half:]
    xf = x.float()
    if mode == 0:
        a, b = xf[..., :half], xf[..., half:]
        out = torch.cat([a * c - b * s, b * c + a * s], dim=-1)
    else:
        a, b = xf[..., 0::2], xf[..., 1::2]
        out = torch.stack([a * c - b * s, b * c + a * s], dim=-1).flatten(-2)
    return out.to(x.dtype)


def to_cache(x: torch.Tensor, dtype) -> torch.Tensor:
    """K / V rows in the cache's element type: e4m3 caches saturate to +-448 first (the
    kernels' rounding, common.h kv_store*); torch's own cast turns overflow into NaN."""
    if dtype == torch.float8_e4m3fn:
        return x.float().clamp(-448.0, 448.0).to(dtype)
    return x.to(dtype)


def rope_cache(qkv, positions, slots, cos_sin, k_cache, v_cache, nq, nkv, D, mode):
    """In-place: rotates q inside qkv, writes rotated k and raw v into the caches."""
    T = qkv.shape[0]
    if T == 0:
        return
    q = qkv[:, : nq * D].view(T, nq, D)
    k = qkv[:, nq * D:(nq + nkv) * D].view(T, nkv, D)
    v = qkv[:, (nq + nkv) * D:(nq + 2 * nkv) * D].view(T, nkv, D)
    q.copy_(apply_rope(q, positions[:T], cos_sin, mode))
    kr = apply_rope(k, positions[:T], cos_sin, mode)
    bs = k_cache.shape[2]
    sl = slots[:T].long()
    valid = sl >= 0
    if valid.any():
        sv = sl[valid]
        blk, off = sv // bs, sv % bs
        k_cache[blk, :, off, :] = to_cache(kr[valid], k_cache.dtype)
        v_cache[blk, :, :, off] = to_cache(v[valid], v_cache.dtype)


def _gather_kv(k_cache, v_cache, block_table, n):
    bs = k_cache.shape[2]
    idx = torch.arange(n, device=k_cache.device)
    blk = block_table[(idx // bs)].long()
    off = idx % bs
    k = k_cache[blk, :, off, :]          # [n, nkv, D]
    v = v_cache[blk, :, :, off]          # [n, nkv, D]
    return k, v


def paged_decode(q, k_cache, v_cache, block_tables, context_lens, nq, nkv, scale, window=0):
    """q [B, nq*D (+extra)] -> out [B, nq, D] (fp32 math). window > 0: only the
    last ``window`` keys (sliding-window layers)."""
    D = k_cache.shape[3]
    B = context_lens.shape[0]
    G = nq // nkv
    out = torch.empty(B, nq, D, dtype=q.dtype, device=q.device)
    for b in range(B):
        n = int(context_lens[b])
        k, v = _gather_kv(k_cache, v_cache, block_tables[b], n)
        if window > 0 and n > window:
            k, v = k[n - window:], v[n - window:]
        qb = q[b, : nq * D].view(nq, D).float()
        kf = k.float().repeat_interleave(G, dim=1)  # [n, nq, D]
        vf = v.float().repeat_interleave(G, dim=1)
        s = torch.einsum("hd,nhd->hn", qb, kf) * scale
        p = torch.softmax(s, dim=-1)
        out[b] = torch.einsum("hn,nhd->hd", p, vf).to(q.dtype)
    return out


def prefill_attention(q, k_cache, v_cache, block_tables, cu_q, ctx_lens, nq, nkv, scale, window=0):
    """q [T, nq*D (+extra)] -> out [T, nq, D]; causal over absolute positions;
    window > 0: keys within ``window - 1`` positions before the query."""
    D = k_cache.shape[3]
    G = nq // nkv
    T = int(cu_q[-1])
    out = torch.empty(T, nq, D, dtype=q.dtype, device=q.device)
    for s_ in range(len(ctx_lens)):
        q0, q1 = int(cu_q[s_]), int(cu_q[s_ + 1])
        ql, ctx = q1 - q0, int(ctx_lens[s_])
        if ql == 0:
            continue
        k, v = _gather_kv(k_cache, v_cache, block_tables[s_], ctx)
        qs = q[q0:q1, : nq * D].view(ql, nq, D).float()
        kf = k.float().repeat_interleave(G, dim=1)
        vf = v.float().repeat_interleave(G, dim=1)
        s = torch.einsum("qhd,nhd->hqn", qs, kf) * scale
        qpos = torch.arange(ctx - ql, ctx, device=q.device)[:, None]
        kpos = torch.arange(ctx, device=q.device)[None, :]
        mask = kpos > qpos
        if window > 0:
            mask = mask | (kpos <= qpos - window)
        s = s.masked_fill(mask[None], float("-inf"))
        p = torch.softmax(s, dim=-1)
        out[q0:q1] = torch.einsum("hqn,nhd->qhd", p, vf).to(q.dtype)
    return out


# ---- sampling: the same counter-based RNG as csrc/kernels/sampling.hip ----


def row_key(seed: int, step: int) -> int:
    M = (1 << 64) - 1
    x = ((seed & M) * 0x9E3779B97F4A7C15 & M) ^ (((step & M) + 0xD1B54A32D192ED03) & M) * 0xBF58476D1CE4E5B9 & M
    x ^= x >> 31
    x = x * 0x7FB5D329728EA185 & M
    x ^= x >> 27
    x = x * 0x81DADEF4BC2DD44D & M
    x ^= x >> 33
    return (x ^ (x >> 32)) & 0xFFFFFFFF


def uniform01(seed: int, step: int, n: int) -> np.ndarray:
    key = np.uint32(row_key(seed, step))
    with np.errstate(over="ignore"):
        i = np.arange(n, dtype=np.uint32)
        h = key ^ (i * np.uint32(0x9E3779B9) + np.uint32(0x7F4A7C15))
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    return (((h >> np.uint32(8)).astype(np.float64) + 0.5) / 16777216.0).astype(np.float32)


def sample(logits: torch.Tensor, temperature, top_k, top_p, seeds, steps, bf16_row: bool = True):
    """Returns (tokens int64 [B], logprobs f32 [B]) with the kernel's semantics:
    greedy if T<=1e-5; else top-k then top-p (on the top-k-renormalised mass) then
    a Gumbel-max draw with u = hash(seed, step, index). ``bf16_row`` mirrors the
    kernel, which holds an fp32 row as bf16; the CPU engine samples full fp32."""
    B, V = logits.shape
    toks = torch.empty(B, dtype=torch.long)
    lps = torch.empty(B, dtype=torch.float32)
    # the kernel holds the row as bf16 in registers: sample on bf16-rounded logits
    lf = logits.float().cpu()
    if bf16_row:
        lf = lf.to(torch.bfloat16).float()
    for r in range(B):
        x = lf[r]
        lse = torch.logsumexp(x, 0)
        t = float(temperature[r])
        if not t > 1e-5:
            i = int(torch.argmax(x))
            toks[r], lps[r] = i, float(x[i] - lse)
            continue
        keep = torch.ones(V, dtype=torch.bool)
        k = int(top_k[r])
        if 0 < k < V:
            kth = torch.topk(x, k).values[-1]
            keep &= x >= kth
        p = float(top_p[r])
        if p < 1.0:
            w = torch.exp((x - x.max()) / t) * keep
            order = torch.argsort(x, descending=True)
            cum = torch.cumsum(w[order].double(), 0)
            target = p * float(cum[-1])
            n = int(torch.searchsorted(cum, torch.tensor([target], dtype=torch.float64))[0])
            thr = x[order[min(n, V - 1)]]
            keep &= x >= thr
        u = torch.from_numpy(uniform01(int(seeds[r]), int(steps[r]), V))
        g = (x - x.max()) / t - torch.log(-torch.log(u))
        g = torch.where(keep, g, torch.full_like(g, float("-inf")))
        i = int(torch.argmax(g))
        toks[r], lps[r] = i, float(x[i] - lse)
    return toks, lps


# ----------------------------------------------------------------------------- K16
def _mix32(x: torch.Tensor) -> torch.Tensor:
    """lowbias32 on int64 tensors holding uint32 values (products wrap mod 2^64,
    the low 32 bits are exact)."""
    M = 0xFFFFFFFF
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & M
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & M
    return x ^ (x >> 16)


def fill_uniform(out: torch.Tensor, row0: int, col0: int, gcols: int, key: int, scale: float):
    """Torch twin of csrc/kernels/init.hip (bit-identical): uniform(-scale, scale)
    keyed by global element coordinates, written into the 2-D view ``out``."""
    rows, cols = out.shape
    r = torch.arange(rows, dtype=torch.int64).unsqueeze(1) + row0
    c = torch.arange(cols, dtype=torch.int64).unsqueeze(0) + col0
    idx = (r * gcols + c) & 0xFFFFFFFF
    h = _mix32(_mix32(idx) ^ (key & 0xFFFFFFFF))
    u = (h >> 8).to(torch.float32) * 5.9604644775390625e-08
    v = (u - 0.5) * torch.tensor(2.0 * scale, dtype=torch.float32)
    out.copy_(v.to(torch.bfloat16).to(out.dtype))
    return out


# ---------------------------------------------------------------- penalties / logprobs
# Oracle of csrc/kernels/penalties.hip. State per slot: counts int32 [slots, V]
# (generated-token occurrences), seen int32 [slots, ceil(V/32)] bitmask (prompt or
# generated). vLLM / OpenAI order: repetition first, then frequency + presence.
def _seen_mask(seen: torch.Tensor, V: int) -> torch.Tensor:
    v = torch.arange(V, device=seen.device)
    return ((seen[:, v // 32] >> (v % 32)) & 1).bool()


def penalty_apply(logits, slot, pres, freq, rep, counts, seen):
    rows, V = logits.shape
    for r in range(rows):
        s = int(slot[r])
        p, f, q = float(pres[r]), float(freq[r]), float(rep[r])
        if s < 0 or (p == 0.0 and f == 0.0 and q == 1.0):
            continue
        l = logits[r].float()
        m = _seen_mask(seen[s:s + 1], V)[0]
        l = torch.where(m, torch.where(l > 0, l / q, l * q), l)
        c = counts[s].float()
        l = l - f * c - p * (c > 0).float()
        logits[r].copy_(l.to(logits.dtype))
    return logits


def penalty_update(tok, slot, counts, seen):
    V = counts.shape[1]
    for r in range(tok.shape[0]):
        s, t = int(slot[r]), int(tok[r])
        if s < 0 or not 0 <= t < V:
            continue
        counts[s, t] += 1
        seen[s, t // 32] |= _bit(t)


def _bit(t: int) -> int:
    b = 1 << (t % 32)
    return b - (1 << 32) if b >= (1 << 31) else b  # int32 two's complement


def penalty_init(counts, seen, slots, off, n_prompt, toks):
    V = counts.shape[1]
    for j in range(slots.shape[0]):
        s = int(slots[j])
        counts[s].zero_()
        seen[s].zero_()
        a, b, npr = int(off[j]), int(off[j + 1]), int(n_prompt[j])
        for i in range(a, b):
            t = int(toks[i])
            if not 0 <= t < V:
                continue
            seen[s, t // 32] |= _bit(t)
            if i - a >= npr:
                counts[s, t] += 1


def top_logprobs(logits, nreq, out_ids, out_lp):
    """n largest log-softmax entries per row (ties -> lowest id), K = out width.

    Exact over the whole row. The device kernel (csrc/kernels/penalties.hip
    top_logprobs) is exact too unless more than 64 keys share the bf16 bin of the n-th
    largest value: it then keeps the lowest-index 64 of them, so in a row
    with > 64 logits within one bf16 ulp of the n-th largest the two may name different
    (equally probable to bf16 precision) entries."""
    K = out_ids.shape[1]
    out_ids.fill_(-1)
    out_lp.fill_(float("-inf"))
    for r in range(logits.shape[0]):
        n = min(int(nreq[r]), K)
        if n <= 0:
            continue
        l = logits[r].float()
        ls = l - torch.logsumexp(l, 0)
        # order by (exact value desc, id asc): stable sort keeps equal values in id order
        order = torch.argsort(-l, stable=True)[:n].tolist()
        for i, v in enumerate(order):
            out_ids[r, i] = v
            out_lp[r, i] = ls[v]
