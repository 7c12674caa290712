"""Quantised (GGUF) weights on the GPU and the matmul that consumes them.

``QuantWeight`` repacks GGUF blocks once at load into the layouts
``csrc/kernels/gguf.hip`` reads with aligned 16-byte loads (K-quants stay in their
native super-blocks, Q6_K is padded to 224 B, Q8_0/Q4_0/Q4_1 become
structure-of-arrays) and keeps merged projections (q|k|v, gate|up) as parts that
may use different formats (Q4_K_M puts attn_v/ffn_down in Q6_K).

``quant_linear(x, w)``: decode batches (M <= 64) run the fused dequant-in-register
f16-MFMA GEMM of ``csrc/kernels/gguf_mfma.hip`` — ONE launch per format over all
parts of a merged projection (256 weight rows per workgroup, split-K for
occupancy); ``quant_partial`` hands its fp32 split-K partials to the fused decode
epilogues (RoPE + KV write, residual + RMSNorm, GLU). Larger M (prefill)
dequantises every part into one contiguous bf16 scratch and runs ONE hipBLASLt
GEMM.
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..weights import gguf as G

# FP8 e4m3 weights (compressed-tensors "FP8-Dynamic" per-channel / per-tensor scales,
# and 128 x 128 block-scaled FP8) share the v2 kernel: pseudo type ids beside ggml's
FP8, FP8B = 1000, 1001
# 8-bit integer weight-only (compressed-tensors pack-quantized 8-bit / AWQ 8-bit):
# unsigned bytes u = q + 128, per-group scale and zero point
INT8 = 1002
# per-channel symmetric 8-bit (one scale per row, no zero point): the bytes alone in the
# tiled layout, the scale as the fp32 row scale ``rs`` (gguf_tiles.h INT8C)
INT8C = 1003
KERNEL_QT = {G.Q4_0: 0, G.Q4_1: 1, G.Q8_0: 2, G.Q4_K: 3, G.Q5_K: 4, G.Q6_K: 5, FP8: 6, FP8B: 7, INT8: 8,
             INT8C: 9}
MAX_FUSED_M = 64
# the W8A8 FP8 decode GEMM (fp8_decode.hip) also takes the decode graph buckets above 64
# rows (up to 256, max_num_seqs' default): one weight stream per step instead of the
# prefill GEMM, which left most of the chip idle at these row counts — Gemma-3-27B FP8 at
# 256 sequences: 35.2 ms of FP8 GEMMs per decode step (0.8 TB/s)
F8_DECODE_MAX_M = 256
# prefill chunks up to this many tokens without a bf16 shadow run the dequant-MFMA
# kernel swept over 64-row M tiles (K15: no [N, K] bf16 dequant pass, which costs more
# than the GEMM itself at small M); larger chunks dequantise into scratch + hipBLASLt.
# Llama-3-8B Q4_K gate|up (profiles/r2_k15_prefill_quant_gemm.jsonl): M = 128: 65 us vs
# 150 dequant + hipBLASLt; M = 512: equal; a resident bf16 shadow beats both (41 / 93 us)
QPREFILL_MAX_M = int(os.environ.get("HIPSERVE_QPREFILL_MAX_M", "512"))


def repack(raw: np.ndarray, qtype: int, N: int, K: int):
    """GGUF raw bytes of an [N, K] matrix -> (q uint8 [N, row_bytes], d, m, row_bytes)."""
    be, bb = G.BLOCK[qtype]
    nb = K // be
    b = np.asarray(raw, np.uint8).reshape(N, nb, bb)
    empty = np.zeros(0, np.uint16)
    if qtype in (G.Q4_K, G.Q5_K):
        q = b.reshape(N, nb * bb)
        return q, empty, empty, nb * bb
    if qtype == G.Q6_K:
        q = np.zeros((N, nb, 224), np.uint8)
        q[:, :, :210] = b
        return q.reshape(N, nb * 224), empty, empty, nb * 224
    if qtype == G.Q8_0:
        d = b[:, :, 0:2].copy().view(np.uint16).reshape(N, nb)
        q = b[:, :, 2:34].reshape(N, K)
        return q, d, empty, K
    if qtype == G.Q4_0:
        d = b[:, :, 0:2].copy().view(np.uint16).reshape(N, nb)
        q = b[:, :, 2:18].reshape(N, K // 2)
        return q, d, empty, K // 2
    if qtype == G.Q4_1:
        d = b[:, :, 0:2].copy().view(np.uint16).reshape(N, nb)
        m = b[:, :, 2:4].copy().view(np.uint16).reshape(N, nb)
        q = b[:, :, 4:20].reshape(N, K // 2)
        return q, d, m, K // 2
    raise NotImplementedError(G.TYPE_NAMES.get(qtype, qtype))


CHUNK_BYTES = {G.Q4_K: 2304, G.Q5_K: 2816, G.Q6_K: 3360, G.Q8_0: 4352, G.Q4_0: 2304, G.Q4_1: 2560,
               FP8: 4096, FP8B: 4224, INT8: 4608, INT8C: 4096}


def _lanes(a: np.ndarray, n_ld: int) -> np.ndarray:
    """[R, nsb, 16 rows, 4 g, n_ld, 16 B] -> [R, nsb, n_ld * 64 lanes * 16 B]: load j of
    lane 16 g + c at j * 1024 + 16 * lane (one coalesced 1 KiB access per load)."""
    R, nsb = a.shape[:2]
    return a.transpose(0, 1, 4, 3, 2, 5).reshape(R, nsb, n_ld * 1024)


def repack_tiled(raw: np.ndarray, qtype: int, N: int, K: int) -> np.ndarray:
    """GGUF raw bytes of an [N, K] matrix (N % 16 == 0, K % 256 == 0) -> the v2
    decode kernel's tiled layout uint8 [N/16, K/256, chunk] (csrc/kernels/gguf_mfma.hip):
    each chunk holds the 16 rows x 256 k one wave multiplies, lane-interleaved."""
    be, bb = G.BLOCK[qtype]
    R, nsb = N // 16, K // 256
    per = 256 // be                      # ggml blocks per 256-k super-chunk
    b = np.asarray(raw, np.uint8).reshape(R, 16, nsb, per * bb).transpose(0, 2, 1, 3)  # [R, nsb, 16, bytes]
    if qtype in (G.Q4_K, G.Q5_K):
        qo = 16 if qtype == G.Q4_K else 48
        parts = [b[..., 0:16].reshape(R, nsb, 256),
                 _lanes(b[..., qo:qo + 128].reshape(R, nsb, 16, 4, 2, 16), 2)]
        if qtype == G.Q5_K:
            parts.append(b[..., 16:48].reshape(R, nsb, 512))
    elif qtype == G.Q6_K:
        parts = [_lanes(b[..., 0:128].reshape(R, nsb, 16, 4, 2, 16), 2),
                 b[..., 128:192].reshape(R, nsb, 1024), b[..., 192:208].reshape(R, nsb, 256),
                 b[..., 208:210].reshape(R, nsb, 32)]
    else:
        blk = b.reshape(R, nsb, 16, per, bb)
        if qtype == G.Q8_0:
            q = blk[..., 2:34].reshape(R, nsb, 16, 4, 4, 16)       # lane g: bytes 64 g + 16 i
            parts = [_lanes(q, 4), blk[..., 0:2].reshape(R, nsb, 256)]
        else:
            qo = 2 if qtype == G.Q4_0 else 4
            q = blk[..., qo:qo + 16].reshape(R, nsb, 16, 4, 2, 16)  # lane g: blocks 2g, 2g+1
            parts = [_lanes(q, 2), blk[..., 0:2].reshape(R, nsb, 256)]
            if qtype == G.Q4_1:
                parts.append(blk[..., 2:4].reshape(R, nsb, 256))
    out = np.concatenate(parts, axis=2)
    assert out.shape[2] == CHUNK_BYTES[qtype]
    return np.ascontiguousarray(out)


# gguf_mfma.hip places each quantised integer at bit SUB_SHIFT of a subnormal f16 and
# scales it by 2^(24 - SUB_SHIFT) inside the f16 FMA: every block scale must stay below
# 65504 / 2^(24 - SUB_SHIFT) (|w| up to ~2-4). Weights beyond that (none in practice)
# run on the v1 kernel.
SUB_SHIFT = {G.Q4_K: 6, G.Q5_K: 5, G.Q6_K: 4, G.Q8_0: 2, G.Q4_0: 6, G.Q4_1: 6}


def sub_scale_ok(raw, qtype: int) -> bool:
    if qtype not in SUB_SHIFT:
        return True
    lim = 65504.0 / 2.0 ** (24 - SUB_SHIFT[qtype])
    _, bb = G.BLOCK[qtype]
    b = np.asarray(raw, np.uint8).reshape(-1, bb)

    def f16(a):
        return np.abs(np.ascontiguousarray(a).view(np.float16).astype(np.float32).reshape(-1))
    if qtype in (G.Q4_K, G.Q5_K):
        sc, _ = G._scale_min_k4(b[:, 4:16])
        prod = f16(b[:, 0:2])[:, None] * sc
    elif qtype == G.Q6_K:
        prod = f16(b[:, 208:210])[:, None] * np.abs(np.ascontiguousarray(b[:, 192:208]).view(np.int8).astype(np.float32))
    else:
        prod = f16(b[:, 0:2])[:, None]
    # (no lower bound: a d * sc below the f16 normal range is kept with MORE mantissa
    # bits than the magic-number path's f16-subnormal scale — see gguf_mfma.hip)
    return bool(prod.size == 0 or np.max(prod) < lim)


def tileable(N: int, K: int) -> bool:
    return N % 16 == 0 and K % 256 == 0


class QuantPart:
    """One quantised matrix on the device: ``tiled`` parts (N % 16 == 0) hold the v2
    layout in ``q`` [N/16, K/256, chunk]; others (GGUF only) the v1 row layout + SoA
    scales. FP8 parts carry ``rs``, the fp32 per-row output scale (256 x the
    channel scale: the kernel's e4m3 -> f16 bit move yields value / 256)."""

    def __init__(self, qtype, N, K, q, d, m, row_bytes, tiled=False, rs=None, sub_ok=True):
        self.qtype, self.N, self.K = qtype, N, K
        self.kqt = KERNEL_QT[qtype]
        self.q, self.d, self.m, self.row_bytes = q, d, m, row_bytes
        self.tiled = tiled
        self.sub_ok = sub_ok  # block scales in the v2 kernel's subnormal-dequant range
        self.rs = rs if rs is not None else torch.empty(0, dtype=torch.float32, device=q.device)

    @classmethod
    def from_int8(cls, u: torch.Tensor, scale: torch.Tensor, zero_point: torch.Tensor | None, device,
                  channel: bool = True):
        """8-bit weight-only matrix: ``u`` [N, K] unsigned bytes holding q + 128 (the
        compressed-tensors pack-quantized convention), ``scale`` [N, K / group] or
        [N, 1] (per channel), optional signed ``zero_point`` of the same shape:
        w = (u - 128 - zp) * scale. Groups of >= 32 k; N % 16 == 0, K % 256 == 0.
        Per-channel scales without a zero point become INT8C unless ``channel`` is False
        (a stack of experts that must share one format)."""
        N, K = u.shape
        u = u.to(device=device, dtype=torch.uint8)
        sc = scale.to(device=device, dtype=torch.float32).reshape(N, -1)
        ng = sc.shape[1]
        G = K // ng
        if G * ng != K or G < 32 or G % 32:
            raise ValueError(f"int8 group size {K}/{ng} not supported (needs a multiple of 32)")
        zp = (zero_point.to(device=device, dtype=torch.float32).reshape(N, -1) if zero_point is not None
              else torch.zeros_like(sc))
        R, nsb = N // 16, K // 256
        lanes = u.reshape(R, 16, nsb, 4, 4, 16).permute(0, 2, 4, 3, 1, 5).reshape(R, nsb, 4096)
        if channel and ng == 1 and (zero_point is None or not bool(zp.any())):
            # per channel, symmetric: INT8C (the bytes alone, the scale applied to the
            # accumulators: 4096 instead of 4608 bytes per 16 x 256 chunk)
            return cls(INT8C, N, K, lanes.contiguous(), _E16(device), _E16(device), 0, tiled=True,
                       rs=sc.reshape(N).contiguous())
        # (scale, offset = -(1024 + 128 + zp)) per (row, super-chunk, lane quarter g, half h): k0 = 256 sb + 64 g + 32 h
        k0 = torch.arange(nsb * 8, device=device) * 32                 # [nsb * 4 * 2] in (sb, g, h) order
        gi = k0 // G
        s16 = sc[:, gi].to(torch.float16)                              # [N, nsb*8]
        o16 = (-(1152.0 + zp[:, gi])).to(torch.float16)
        meta = torch.stack([s16, o16], -1).reshape(R, 16, nsb, 8, 2).permute(0, 2, 1, 3, 4).contiguous()
        chunk = torch.cat([lanes, meta.view(torch.uint8).reshape(R, nsb, 512)], 2).contiguous()
        return cls(INT8, N, K, chunk, _E16(device), _E16(device), 0, tiled=True)

    @classmethod
    def from_fp8(cls, q: torch.Tensor, scale: torch.Tensor, device):
        """FP8 e4m3 weight [N, K] (float8_e4m3fn or its uint8 bits) and its scale:
        one value (per tensor), [N] / [N, 1] (per output channel) or
        [ceil(N/128), ceil(K/128)] (128 x 128 blocks). N % 16 == 0, K % 256 == 0."""
        N, K = q.shape
        q = q.to(device)
        q8 = q.view(torch.uint8) if q.dtype != torch.uint8 else q
        s = scale.to(device=device, dtype=torch.float32)
        R, nsb = N // 16, K // 256
        lanes = q8.reshape(R, 16, nsb, 4, 4, 16).permute(0, 2, 4, 3, 1, 5).reshape(R, nsb, 4096)
        if s.numel() == 1 or (s.numel() == N and (s.dim() == 1 or s.shape[-1] == 1)):
            rs = (256.0 * s.reshape(-1).expand(N)).contiguous()
            return cls(FP8, N, K, lanes.contiguous(), _E16(device), _E16(device), 0, tiled=True, rs=rs)
        bn, bk = s.shape
        if bn * 128 < N or bk * 128 < K:
            raise ValueError(f"block scale {tuple(s.shape)} does not cover a {N}x{K} weight in 128-blocks")
        rows = s[torch.arange(N, device=device) // 128][:, : K // 128]          # [N, K/128]
        blk = rows.reshape(R, 16, nsb, 2).permute(0, 2, 1, 3).contiguous().view(torch.uint8).reshape(R, nsb, 128)
        chunk = torch.cat([lanes, blk], 2).contiguous()
        rs = torch.full((N,), 256.0, dtype=torch.float32, device=device)
        return cls(FP8B, N, K, chunk, _E16(device), _E16(device), 0, tiled=True, rs=rs)

    @classmethod
    def build(cls, raw, qtype: int, N: int, K: int, device):
        def to(a, dt):
            return torch.from_numpy(np.array(a, copy=True, order='C')).view(dt).to(device)
        if tileable(N, K):
            e = torch.empty(0, dtype=torch.int16, device=device)
            return cls(qtype, N, K, to(repack_tiled(raw, qtype, N, K), torch.uint8), e, e, 0, tiled=True,
                       sub_ok=sub_scale_ok(raw, qtype))
        q, d, m, rb = repack(raw, qtype, N, K)
        return cls(qtype, N, K, to(q, torch.uint8), to(d, torch.int16), to(m, torch.int16), rb)

    @property
    def nbytes(self):
        return self.q.numel() + 2 * (self.d.numel() + self.m.numel()) + 4 * self.rs.numel()


class QuantWeight:
    def __init__(self, parts: list[QuantPart]):
        self.parts = parts
        self.N = sum(p.N for p in parts)
        self.K = parts[0].K
        assert all(p.K == self.K for p in parts)
        self._gkey = None
        self.dense = None  # bf16 [N, K] copy for prefill GEMMs (make_dense_shadows), or None

    @property
    def groups(self):
        """One decode-GEMM launch per format: [(kernel qtype, parts, output column of
        each part)] (recomputed if ``parts`` is edited)."""
        key = tuple(map(id, self.parts))
        if key != self._gkey:
            groups: dict[int, tuple[list, list]] = {}
            off = 0
            for p in self.parts:
                ps, cols = groups.setdefault(p.kqt, ([], []))
                ps.append(p)
                cols.append(off)
                off += p.N
            self._groups = [(kqt, ps, cols) for kqt, (ps, cols) in groups.items()]
            self._v2 = all(p.tiled and p.sub_ok for p in self.parts)
            cols = np.cumsum([0] + [p.N for p in self.parts])[:-1].tolist()
            self.v2_args = ([p.q for p in self.parts], [p.rs for p in self.parts], [p.kqt for p in self.parts],
                            [p.N for p in self.parts], cols)
            self._gkey = key
        return self._groups

    @property
    def v2(self) -> bool:
        """The v2 MFMA kernel applies (every part tiled), unless disabled."""
        self.groups
        return self._v2 and not getattr(self, "_v2_off", False)

    @v2.setter
    def v2(self, on: bool):
        self._v2_off = not on

    @property
    def shape(self):
        return (self.N, self.K)

    @property
    def nbytes(self):
        return sum(p.nbytes for p in self.parts)

    @staticmethod
    def supported(qtype: int, K: int) -> bool:
        return qtype in KERNEL_QT and K % 256 == 0

    @classmethod
    def from_gguf(cls, gf: "G.GGUFFile", names, device):
        parts = []
        for n in names:
            t = gf.tensors[n]
            N, K = t.rows_cols
            if not cls.supported(t.type, K):
                return torch.cat([torch.from_numpy(gf.tensor_f32(x)).to(device, torch.bfloat16)
                                  for x in names], 0)
            parts.append(QuantPart.build(gf.raw(n), t.type, N, K, device))
        return cls(parts)

    @classmethod
    def from_raw(cls, raws: list, device):
        """[(qtype, N, K, raw ggml bytes)] -> QuantWeight on ``device``."""
        return cls([QuantPart.build(raw, qtype, N, K, device) for qtype, N, K, raw in raws])

    @classmethod
    def from_float(cls, w: np.ndarray | list, qtype: int, device):
        """Quantise float matrices (tests / synthetic benchmarks)."""
        mats = w if isinstance(w, list) else [w]
        parts = []
        for mat in mats:
            mat = np.asarray(mat, np.float32)
            N, K = mat.shape
            parts.append(QuantPart.build(G.quantize(mat, qtype), qtype, N, K, device))
        return cls(parts)


# synthetic block scales: |w| ~ 0.02 for every format (random-init benchmarks)
_SYNTH_D = {G.Q4_K: (8e-5, 6e-4), G.Q5_K: (4e-5, 6e-4), G.Q6_K: (1.5e-5, 0.0), G.Q8_0: (2.5e-4, 0.0),
            G.Q4_0: (4e-3, 0.0), G.Q4_1: (4e-3, -0.03)}


def random_blocks(rng: np.random.Generator, qtype: int, N: int, K: int) -> np.ndarray:
    """Random GGUF blocks of an [N, K] matrix in ggml's raw layout: random quant
    bits and sub-block scales, fixed per-block fp16 scale(s) — valid blocks of the
    real format without quantising float weights (an 8B model in seconds)."""
    be, bb = G.BLOCK[qtype]
    nb = K // be
    b = rng.integers(0, 256, size=(N, nb, bb), dtype=np.uint8)
    d, dm = _SYNTH_D[qtype]
    f16 = lambda v: np.frombuffer(np.float16(v).tobytes(), np.uint8)  # noqa: E731
    if qtype in (G.Q4_K, G.Q5_K):
        b[:, :, 0:2] = f16(d)
        b[:, :, 2:4] = f16(dm)
    elif qtype == G.Q6_K:
        b[:, :, 208:210] = f16(d)
    elif qtype in (G.Q8_0, G.Q4_0, G.Q5_0):
        b[:, :, 0:2] = f16(d)
    elif qtype in (G.Q4_1, G.Q5_1):
        b[:, :, 0:2] = f16(d)
        b[:, :, 2:4] = f16(dm)
    return b.reshape(-1)


_scratch: dict = {}


def _dequant_scratch(device, numel):
    buf = _scratch.get(device)
    if buf is None or buf.numel() < numel:
        buf = torch.empty(numel, dtype=torch.bfloat16, device=device)
        _scratch[device] = buf
    return buf


def _dequant_into(buf: torch.Tensor, p: QuantPart):
    if p.tiled:
        torch.ops.hipserve.gguf_dequant_tiled(buf, p.q, p.rs, p.kqt, p.N, p.K)
    else:
        torch.ops.hipserve.gguf_dequant(buf, p.q, p.d, p.m, p.kqt, p.row_bytes, p.N, p.K)


def dequantize(w: QuantWeight) -> torch.Tensor:
    out = torch.empty(w.N, w.K, dtype=torch.bfloat16, device=w.parts[0].q.device)
    off = 0
    for p in w.parts:
        _dequant_into(out[off:off + p.N], p)
        off += p.N
    return out


def _splits(N: int, K: int) -> int:
    """K slices for the v1 decode dequant-GEMM: ~512 (64-row tile, K slice) workgroups."""
    wgs = (N + 63) // 64
    nsb = K // 256
    return max(1, min(nsb, -(-512 // wgs)))


ROWS_PER_WG = 128      # gguf_mfma.hip: 4 waves x 2 row groups of 16
TARGET_WGS = 1024      # ~4 four-wave workgroups per CU


def _actual_splits(nsb: int, S: int) -> int:
    per = -(-nsb // S)
    return -(-nsb // per)


# (weight signature, M bucket) -> S, measured by tune_splits at engine start
SPLIT_TABLE: dict = {}
M_BUCKETS = (1, 8, 16, 32, 48, 64)
F8_M_BUCKETS = M_BUCKETS + (128, 256)  # split tables of the FP8 decode GEMM
PARTIAL_READ_BPS = 5e12   # the fused epilogue re-reads the fp32 partials at ~HBM rate
COLD_BYTES = 768 << 20    # split timing rotates over block copies of at least this many bytes


def _sig(w: QuantWeight):
    return (w.K, tuple((p.kqt, p.N) for p in w.parts))


def _bucket(M: int) -> int:
    for b in F8_M_BUCKETS:
        if M <= b:
            return b
    return F8_M_BUCKETS[-1]


def v2_splits(w: QuantWeight, M: int) -> int:
    """K slices for the v2 kernel: the tuned choice for (weight shape, M bucket) if
    any, else enough (row tile, K slice) workgroups to fill the chip, capped so the
    fp32 partials (S*M*N*4 B) stay below the weight bytes."""
    S = SPLIT_TABLE.get((_sig(w), _bucket(M)))
    if S is not None:
        return S
    tiles = sum(-(-p.N // ROWS_PER_WG) for _, ps, _ in w.groups for p in ps)
    nsb = w.K // 256
    if tiles >= 512:
        return 1
    S = min(nsb, -(-TARGET_WGS // tiles))
    cap = max(1, w.nbytes // max(1, 4 * M * w.N))
    return _actual_splits(nsb, max(1, min(S, cap)))


_EMPTY: dict = {}


def _E16(device):
    return torch.empty(0, dtype=torch.int16, device=device)


def _empty(device, dtype):
    key = (device, dtype)
    t = _EMPTY.get(key)
    if t is None:
        t = _EMPTY[key] = torch.empty(0, dtype=dtype, device=device)
    return t


def _launch_v2(out, ws, x, w: QuantWeight, S: int, x16=None, qs=None):
    """The v2 kernel with S K slices; ``qs``: other copies of the parts' blocks
    (cold-cache timing)."""
    w.groups  # (re)builds v2_args
    a = w.v2_args
    return torch.ops.hipserve.gguf_gemm_parts(out, ws, x, qs if qs is not None else a[0], a[1], a[2], a[3], a[4],
                                              w.N, w.K, S, x16)


def _graph_time_us(fn, reps: int = 10, rounds: int = 3) -> float:
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    best = float("inf")
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        best = min(best, 1000 * e0.elapsed_time(e1) / reps)
    del g
    return best


@torch.inference_mode()  # like the engine's graph capture: a process may hold several engines, and the
# generator state tensors a capture registers must not switch between inference and normal tensors
def tune_splits(weights, device, ms=M_BUCKETS, max_ws_bytes: int = 256 << 20, f8_ms=None) -> list:
    """Measure the v2 decode GEMM per distinct QuantWeight shape and M bucket for
    S in {1, 2, 4, ...} and keep the S minimising kernel time + the epilogue's
    re-read of the partials (S*M*N*4 B at PARTIAL_READ_BPS). Timed inside a
    hipGraph (the decode step's launch mode). ``f8_ms``: the M buckets of the FP8 W8A8
    decode GEMM's weights (default ``ms``; it also serves buckets above 64 rows).
    Returns report rows."""
    f8_ms = list(ms) if f8_ms is None else list(f8_ms)
    from . import tune_cache as TC

    seen, report = {}, []
    for w in weights:
        if isinstance(w, QuantWeight) and w.v2:
            seen.setdefault(_sig(w), w)
    for sig in list(seen):  # timed by a previous start on this device and kernel build
        kind = "f8_splits" if f8_decode_ok(seen[sig]) else "gguf_splits"
        mlist = f8_ms if kind == "f8_splits" else ms
        hits = [TC.get(device, kind, [list(map(list, sig[1])), sig[0], M]) for M in mlist]
        if all(h is not None for h in hits):
            for M, h in zip(mlist, hits):
                (F8_SPLIT_TABLE if kind == "f8_splits" else SPLIT_TABLE)[(sig, _bucket(M))] = h["S"]
                report.append(dict(h["row"], cached=True))
            del seen[sig]
    nbuf = max((4 * w.N * max(f8_ms if f8_decode_ok(w) else ms) * 32 for w in seen.values()), default=0)
    ws = torch.empty(min(nbuf, max_ws_bytes) // 4, dtype=torch.float32, device=device)
    empty = _empty(device, torch.bfloat16)
    for sig, w in seen.items():
        nsb = w.K // 256
        if f8_decode_ok(w):  # these run the W8A8 FP8 decode GEMM (M <= F8_DECODE_MAX_M)
            report += _tune_f8_decode(w, f8_ms, ws)
            continue
        # cold weights, as in a decode step (every layer's blocks read once from HBM): the
        # timed calls rotate over copies of the blocks totalling >= COLD_BYTES, so the
        # 256 MiB MALL cannot serve them (warm timing favoured the shallow v2 pipeline)
        a = w.v2_args
        ncopy = max(1, min(64, -(-COLD_BYTES // max(1, w.nbytes))))
        copies = [a[0]] + [[q.clone() for q in a[0]] for _ in range(ncopy - 1)]
        for M in ms:
            x = torch.randn(M, w.K, device=device, dtype=torch.bfloat16)
            # at 33-64 rows the decode producers hand the GEMM an f16 pair-order copy of x
            # (out16 / act16), staged as is: time that form
            x16 = x.to(torch.float16) if 32 < M <= 64 else None
            cands = sorted({_actual_splits(nsb, s) for s in (1, 2, 4, 8, 16, 32, 64) if s <= nsb})
            cost = {}
            for S in cands:
                if S * M * w.N > ws.numel():
                    continue
                t = _graph_time_us(lambda S=S: [_launch_v2(empty, ws, x, w, S, x16, qs) for qs in copies],
                                   reps=max(1, 10 // ncopy)) / ncopy
                cost[S] = t + 1e6 * S * M * w.N * 4 / PARTIAL_READ_BPS
            best = min(cost, key=cost.get)
            SPLIT_TABLE[(sig, _bucket(M))] = best
            row = {"K": w.K, "N": w.N, "M": M, "S": best, "us": {k: round(v, 2) for k, v in sorted(cost.items())}}
            report.append(row)
            TC.put(device, "gguf_splits", [list(map(list, sig[1])), sig[0], M], {"S": best, "row": row})
        del copies
    del ws
    TC.flush()
    return report


# FP8 W8A8 decode (fp8_decode.hip): per-token e4m3 activations x per-channel e4m3
# weights on the scaled FP8 MFMA, no dequant VALU — the FP8-Dynamic checkpoints'
# activation scheme, as the prefill GEMM (ops/pgemm.py f8_gemm). HIPSERVE_FP8_DECODE=0
# keeps the W8A16 v2 kernel (f16 activations).
F8_DECODE = os.environ.get("HIPSERVE_FP8_DECODE", "1") != "0"
F8D_STEPS = (1, 2, 3, 4, 6, 7, 8, 12, 14, 16, 21)  # (K / 256) / S the kernel is built for
F8D_MIN_WGS = 160  # untuned default; measured at 64 rows, 170-250 workgroups of 8 waves stream best


def f8_decode_ok(w) -> bool:
    """The FP8 decode GEMM takes ``w``: per-channel FP8 parts only (no 128-block
    scales), tiled, at most 4 parts, and a K whose 256-k steps split into a built
    step count."""
    parts = getattr(w, "parts", None)
    if not (F8_DECODE and parts and len(parts) <= 4 and hasattr(torch.ops.hipserve, "fp8_decode_gemm")):
        return False
    if not all(p.qtype == FP8 and p.tiled and p.N % 16 == 0 for p in parts) or w.K % 256:
        return False
    return f8_decode_splits(w, 64) > 0


F8_SPLIT_TABLE: dict = {}  # (weight signature, M bucket) -> S, measured by tune_splits


def _f8_valid_splits(w) -> list:
    tiles, nsb = -(-w.N // 128), w.K // 256
    return [S for S in range(1, nsb + 1) if nsb % S == 0 and nsb // S in F8D_STEPS and tiles * S <= 1024]


def f8_decode_splits(w, M: int) -> int:
    """K slices: the tuned choice for (weight shape, M bucket) if any, else the smallest
    S (with (K/256)/S a built step count) giving >= F8D_MIN_WGS workgroups of 128 rows,
    else the largest one under 1024; 0 if none."""
    S = F8_SPLIT_TABLE.get((_sig(w), _bucket(M)))
    if S is not None:
        return S
    tiles, nsb = -(-w.N // 128), w.K // 256
    valid = [S for S in range(1, nsb + 1) if nsb % S == 0 and nsb // S in F8D_STEPS]
    if not valid:
        return 0
    for S in valid:
        if tiles * S >= F8D_MIN_WGS:
            return S
    under = [S for S in valid if tiles * S <= 1024]
    return max(under) if under else valid[0]


def f8_decode_partial(x: torch.Tensor, w: QuantWeight, x8=None):
    """(fp32 split-K partials [S, M, N], S) of x @ w.T, W8A8 (x quantised per token;
    ``x8``: its (e4m3, scales) already written by the producer)."""
    from . import pgemm
    M = x.shape[0]
    xq, xs = x8 if x8 is not None else pgemm.act_quant(x)
    S = f8_decode_splits(w, M)
    ws = torch.empty(S * M * w.N, dtype=torch.float32, device=x.device)
    torch.ops.hipserve.fp8_decode_gemm(ws, xq, xs, [p.q for p in w.parts], [p.rs for p in w.parts], S)
    return ws, S


def _tune_f8_decode(w, ms, ws) -> list:
    """F8_SPLIT_TABLE for one weight shape: each valid S timed in a hipGraph per M
    bucket, plus the epilogue's re-read of the partials (as tune_splits)."""
    from . import pgemm
    rows = []
    for M in ms:
        x = torch.randn(M, w.K, device=ws.device, dtype=torch.bfloat16)
        xq, xs = pgemm.act_quant(x)
        qs, rs = [p.q for p in w.parts], [p.rs for p in w.parts]
        cost = {}
        for S in _f8_valid_splits(w):
            if S * M * w.N > ws.numel():
                continue
            t = _graph_time_us(lambda S=S: torch.ops.hipserve.fp8_decode_gemm(ws, xq, xs, qs, rs, S))
            cost[S] = t + 1e6 * S * M * w.N * 4 / PARTIAL_READ_BPS
        if cost:
            best = min(cost, key=cost.get)
            F8_SPLIT_TABLE[(_sig(w), _bucket(M))] = best
            row = {"K": w.K, "N": w.N, "M": M, "S": best, "kernel": "fp8_w8a8",
                   "us": {k: round(v, 2) for k, v in sorted(cost.items())}}
            rows.append(row)
            from . import tune_cache as TC
            TC.put(ws.device, "f8_splits", [list(map(list, _sig(w)[1])), w.K, M], {"S": best, "row": row})
    return rows


def quant_partial(x: torch.Tensor, w: QuantWeight, x16: torch.Tensor | None = None, x8=None):
    """Decode GEMM writing fp32 split-K partials ws[S, M, N] for a fused epilogue
    (splitk_rope_cache / splitk_add_rmsnorm / splitk_glu); returns (ws, S). ``x16``:
    the producer's f16 pair-order copy of x (splitk_add_rmsnorm / splitk_glu
    ``out16``), staged as is instead of converting x in every workgroup."""
    M = x.shape[0]
    if M <= F8_DECODE_MAX_M and f8_decode_ok(w):
        return f8_decode_partial(x, w, x8)
    S = v2_splits(w, M)
    ws = torch.empty(S * M * w.N, dtype=torch.float32, device=x.device)
    _launch_v2(_empty(x.device, torch.bfloat16), ws, x, w, S, x16)
    return ws, S


# Prefill (M > MAX_FUSED_M) straight from the tiled GGUF blocks (gguf_mfma.hip qpg_kernel:
# each weight dequantised once per 128-256-token tile, f16 MFMA, store / residual-add / GLU
# epilogues): no resident bf16 shadow and no per-call dequantise-into-scratch pass.
# HIPSERVE_QPREFILL: "1" always, "0" never (dequantise into scratch + hipBLASLt), "auto"
# (default): per weight shape, whichever tune_qprefill timed faster at engine start
# (untimed shapes take the block kernel).
QPREFILL_MODE = os.environ.get("HIPSERVE_QPREFILL", "auto")
QPREFILL = QPREFILL_MODE != "0"
QPF_CHOICE: dict = {}  # weight signature -> the block kernel was faster at start-up
GGUF_KQT = (0, 1, 2, 3, 4, 5)  # kernel qtypes Q4_0 .. Q6_K


def qprefill_ok(w, M: int, glu: bool = False, timed: bool = True) -> bool:
    """The block prefill GEMM takes ``w`` at ``M`` rows: a prefill-sized batch, a GGUF
    QuantWeight without a bf16 shadow whose parts are all tiled with block scales in the
    subnormal-dequant range; ``glu``: exactly two parts (gate, up) of one format;
    ``timed``: and the start-up timing (``auto``) did not prefer dequant + hipBLASLt."""
    if not (QPREFILL and isinstance(w, QuantWeight) and M > MAX_FUSED_M and w.dense is None):
        return False
    if not (w.v2 and w.parts[0].q.is_cuda and all(p.kqt in GGUF_KQT for p in w.parts)
            and hasattr(torch.ops.hipserve, "gguf_prefill")):
        return False
    if glu:
        ps = w.parts
        if not (len(ps) == 2 and ps[0].kqt == ps[1].kqt and ps[0].N == ps[1].N):
            return False
    if timed and QPREFILL_MODE == "auto" and M <= QPREFILL_MAX_M:
        return False  # small chunks: the M-tiled K15 kernel (a 256-token tile would be mostly padding)
    return not (timed and QPREFILL_MODE == "auto" and not QPF_CHOICE.get(_sig(w), True))


def tune_qprefill(weights, device, M: int) -> list:
    """Start-up timing, per distinct GGUF weight shape, of the block prefill GEMM (x
    conversion + qpg_kernel, GLU epilogue for (gate, up) pairs) against dequantise into
    scratch + hipBLASLt (+ silu_and_mul) at M rows; fills QPF_CHOICE for ``auto``."""
    from . import pgemm
    seen, rows = {}, []
    for w in weights:
        if qprefill_ok(w, M, timed=False):
            seen.setdefault(_sig(w), w)
    for sig, w in seen.items():
        x = torch.randn(M, w.K, device=device, dtype=torch.bfloat16)
        glu = qprefill_ok(w, M, glu=True, timed=False)
        act = torch.empty(M, w.N // 2, device=device, dtype=torch.bfloat16)

        def blas():
            y = quant_linear_dequant(x, w)
            if glu:
                torch.ops.hipserve.silu_and_mul(act, y)

        def block():
            qprefill(x, w, 2 if glu else 0)
        t_b = pgemm._time(lambda i: blas())
        t_q = pgemm._time(lambda i: block())
        QPF_CHOICE[sig] = t_q <= t_b
        rows.append({"K": w.K, "N": w.N, "M": M, "glu": glu, "block_ms": round(t_q, 4),
                     "dequant_blas_ms": round(t_b, 4), "block": t_q <= t_b})
        del x, act
    torch.cuda.empty_cache()
    return rows


def _qargs(w: QuantWeight):
    w.groups  # (re)builds v2_args
    a = w.v2_args
    return a[0], a[2], a[3], a[4]


def x_f16_pairs(x: torch.Tensor, K: int):
    """(x16, rsc): x[:, :K] as f16 in the GGUF kernels' pair order with each row scaled by
    1 / rsc[m] (a power of two keeping it inside the f16 range) — the block prefill
    GEMM's operand, converted once per activation."""
    M = x.shape[0]
    x16 = torch.empty(M, K, dtype=torch.float16, device=x.device)
    rsc = torch.empty(M, dtype=torch.float32, device=x.device)
    torch.ops.hipserve.x_f16_pairs(x16, rsc, x)
    return x16, rsc


def qprefill(x: torch.Tensor, w: QuantWeight, epi: int = 0, out: torch.Tensor | None = None) -> torch.Tensor:
    """x @ w.T from the blocks: epi 0 store (into ``out`` or a new [M, N]), 1 residual add
    (``out`` += ...), 2 / 3 SiLU / GELU GLU of the (gate, up) parts into [M, N/2]."""
    M = x.shape[0]
    if out is None:
        out = torch.empty(M, w.N // 2 if epi in (2, 3) else w.N, dtype=torch.bfloat16, device=x.device)
    if x.stride(1) != 1 or x.stride(0) % 8:
        x = x.contiguous()
    x16, rsc = x_f16_pairs(x, w.K)
    if not torch.ops.hipserve.gguf_prefill(out, x16, rsc, *_qargs(w), w.K, epi):
        raise RuntimeError(f"gguf_prefill refused parts {[(p.kqt, p.N) for p in w.parts]} K={w.K} epi={epi}")
    return out


def quant_linear(x: torch.Tensor, w: QuantWeight) -> torch.Tensor:
    M = x.shape[0]
    out = torch.empty(M, w.N, dtype=torch.bfloat16, device=x.device)
    if M == 0:
        return out
    if (M <= MAX_FUSED_M or (M <= F8_DECODE_MAX_M and x.is_cuda and f8_decode_ok(w))) and x.stride(1) == 1 \
            and x.stride(0) % 8 == 0:
        if x.is_cuda and f8_decode_ok(w):  # the fused path's partials, reduced: bit-identical to it
            ws, S = f8_decode_partial(x, w)
            torch.ops.hipserve.splitk_reduce(out, ws, S)
            return out
        if w.v2 and x.is_cuda:
            S = v2_splits(w, M)
            if S == 1:
                _launch_v2(out, _empty(x.device, torch.float32), x, w, 1)
                return out
            ws = torch.empty(S, M, w.N, dtype=torch.float32, device=x.device)
            _launch_v2(_empty(x.device, torch.bfloat16), ws, x, w, S)
            torch.ops.hipserve.splitk_reduce(out, ws, S)
            return out
        off = 0
        for p in w.parts:  # v1: row-layout parts only
            if p.tiled:
                buf = _dequant_scratch(x.device, p.N * p.K)[: p.N * p.K].view(p.N, p.K)
                _dequant_into(buf, p)
                out[:, off:off + p.N] = torch.nn.functional.linear(x, buf)
                off += p.N
                continue
            sp = _splits(p.N, p.K)
            ws = torch.empty(sp, M, p.N, dtype=torch.float32, device=x.device) if sp > 1 else \
                torch.empty(0, dtype=torch.float32, device=x.device)
            torch.ops.hipserve.gguf_gemm(out[:, off:off + p.N], x, p.q, p.d, p.m, p.kqt, p.row_bytes,
                                         p.N, p.K, ws, sp)
            off += p.N
        return out
    from . import pgemm
    if pgemm.f8_use(w, M):  # FP8 W8A8: the scaled e4m3 MFMA from the tiled weights, or hipBLASLt FP8
        return pgemm.f8_gemm(x, w, 0, None if getattr(w, "f8_scale", None) is not None else out)
    if w.dense is not None:  # prefill on the resident bf16 copy: no per-call dequant pass
        return torch.nn.functional.linear(x, w.dense)
    if x.is_cuda and qprefill_ok(w, M):
        return qprefill(x, w, 0, out)
    if w.v2 and x.is_cuda and M <= QPREFILL_MAX_M and x.stride(1) == 1 and x.stride(0) % 8 == 0:
        _launch_v2(out, _empty(x.device, torch.float32), x, w, 1)  # K15: M-tiled dequant-MFMA GEMM
        return out
    return quant_linear_dequant(x, w)


def quant_linear_dequant(x: torch.Tensor, w: QuantWeight) -> torch.Tensor:
    """Prefill: every part dequantised into one contiguous [N, K] bf16 scratch, one GEMM."""
    buf = _dequant_scratch(x.device, w.N * w.K)[: w.N * w.K].view(w.N, w.K)
    off = 0
    for p in w.parts:
        _dequant_into(buf[off:off + p.N], p)
        off += p.N
    return torch.nn.functional.linear(x, buf)



def fp8_plain(p: QuantPart) -> torch.Tensor:
    """The plain [N, K] e4m3 bytes of a per-channel FP8 part (inverse of from_fp8's
    tiled permutation)."""
    R, nsb = p.N // 16, p.K // 256
    return p.q.reshape(R, nsb, 4, 4, 16, 16).permute(0, 4, 1, 3, 2, 5).reshape(p.N, p.K)


# FP8 prefill runs hipBLASLt's FP8 GEMM (torch._scaled_mm, row-wise scales: 2.0-2.4
# PFLOP/s on the Gemma-3-27B shapes vs 1.6-1.9 for the hand-written e4m3 kernel,
# tools/bench_pgemm.py --fp8), which needs the weight as plain row-major e4m3.
# HIPSERVE_FP8_PREFILL_LIB:
#   scratch (default): re-laid out per call from the tiled decode copy into a per-device
#       scratch (fp8_untile, one HBM read + write of the weight's bytes): the tiled copy is
#       the ONLY resident copy (the reference hands 0.90 of HBM to the
#       engine, /root/reference/vllm-models/helm-chart/templates/model-deployments.yaml:35-36)
#   resident: a resident plain copy beside the tiled one while HBM allows
#   0: the hand-written e4m3 kernel on the tiled layout (prefill_gemm_f8)
FP8_LIB = os.environ.get("HIPSERVE_FP8_PREFILL_LIB", "scratch")
_F8_SCRATCH: dict = {}


def make_fp8_plain(weights, device, reserve_bytes: int) -> int:
    """Marks the FP8 projections whose prefill GEMM runs on hipBLASLt (``f8_scale``, the
    [1, N] fp32 channel scales) and, in ``resident`` mode, keeps plain [N, K] e4m3 copies
    while ``reserve_bytes`` of HBM stay free. Returns the resident bytes added."""
    if FP8_LIB not in ("scratch", "resident") or torch.device(device).type != "cuda":
        return 0
    from . import pgemm
    added = 0
    for w in sorted(weights, key=lambda w: -w.N * w.K):
        if getattr(w, "f8_scale", None) is not None or not (pgemm.f8_fits(w) or pgemm.f8_fits(w, glu=True)):
            continue
        if not all(p.qtype == FP8 for p in w.parts):
            continue
        w.f8_scale = (torch.cat([p.rs for p in w.parts]) / 256.0).reshape(1, -1).contiguous()
        need = w.N * w.K
        if FP8_LIB == "resident" and torch.cuda.mem_get_info(device)[0] - need >= reserve_bytes:
            w.f8_plain = torch.cat([fp8_plain(p) for p in w.parts]).view(torch.float8_e4m3fn)
            added += need
    return added


def f8_lib_weight(w):
    """The plain [N, K] e4m3 weight for hipBLASLt's FP8 GEMM: the resident copy, or the
    tiled parts re-laid out now into the device's scratch (valid until the next call on
    the stream); None when ``w`` runs the hand-written kernel."""
    wp = getattr(w, "f8_plain", None)
    if wp is not None or getattr(w, "f8_scale", None) is None:
        return wp
    dev = w.parts[0].q.device
    n = w.N * w.K
    buf = _F8_SCRATCH.get(dev)
    if buf is None or buf.numel() < n:
        buf = _F8_SCRATCH[dev] = torch.empty(n, dtype=torch.uint8, device=dev)
    off = 0
    for p in w.parts:
        torch.ops.hipserve.fp8_untile(buf[off * w.K:(off + p.N) * w.K].view(p.N, p.K), p.q, p.N, p.K)
        off += p.N
    return buf[:n].view(w.N, w.K).view(torch.float8_e4m3fn)


def make_dense_shadows(weights, device, reserve_bytes: int, gguf: bool = True) -> int:
    """Keep a dequantised bf16 copy of quantised projections for the prefill GEMMs
    while ``reserve_bytes`` of HBM stay free (288 GB per MI355X: an 8B GGUF model's
    16 GB of bf16 shadows next to its 4.5 GB of blocks). Decode keeps streaming the
    quantised blocks (the v2 dequant-MFMA kernel: 3.6x fewer bytes); prefill skips the
    per-call dequant pass (~18 GB of HBM traffic per 8K-token Llama-3-8B chunk) and
    runs hipBLASLt on the copy. Largest weights first (lm_head, gate|up, ...). GGUF
    weights only with ``gguf`` (the engine passes HIPSERVE_QUANT_SHADOW=1 /
    extra gguf_dense_shadow; default off: a GGUF model's footprint is its blocks, prefill
    reads them through qpg_kernel or a per-call scratch). Returns the bytes added."""
    if torch.device(device).type != "cuda" or os.environ.get("HIPSERVE_QUANT_SHADOW") == "0":
        return 0  # HIPSERVE_QUANT_SHADOW=0: no bf16 shadow for any format
    from . import pgemm
    added = 0
    for w in sorted(weights, key=lambda w: -w.N * w.K):
        if w.dense is not None or pgemm.f8_fits(w) or pgemm.f8_fits(w, glu=True):
            continue  # FP8 prefill runs on the e4m3 MFMA from the quantised weights
        if not gguf and all(p.kqt in GGUF_KQT for p in w.parts):
            continue  # GGUF: prefill from the blocks or a per-call scratch, no resident copy
        need = w.N * w.K * 2
        free, _ = torch.cuda.mem_get_info(device)
        if free - need < reserve_bytes:
            continue
        w.dense = dequantize(w)
        added += need
    return added


class QuantMoE:
    """The quantised experts of one MoE projection, stacked for the expert GEMM
    (``qmoe_gemm``, gguf_mfma.hip MoE mode): ``q`` uint8 [E, N/16 * K/256 * chunk]
    (each expert in the v2 tiled layout), FP8 row scales ``rs`` [E, N]. INT8
    (compressed-tensors 8-bit, the reference's AWQ-8bit export) and per-channel FP8
    experts; prefill runs bf16 expert GEMMs on ``dense`` (a resident shadow when HBM
    allows, else a per-call dequantised scratch)."""

    KERNEL_QTS = (6, 8, 9)  # FP8 (per-row scale), INT8, INT8C (per-row scale)

    def __init__(self, parts: list, kmajor: bool = False):
        p0 = parts[0]
        assert all(p.kqt == p0.kqt and p.N == p0.N and p.K == p0.K and p.tiled for p in parts)
        self.E, self.N, self.K, self.kqt = len(parts), p0.N, p0.K, p0.kqt
        self.q = torch.stack([p.q.reshape(-1) for p in parts]).contiguous()
        # kmajor: each expert [K/256][N/16][chunk] instead of [N/16][K/256][chunk] — at a
        # given super-chunk the workgroups of an expert stream one contiguous column of it
        # (w13 at 64 tokens: 84 -> 72 us, profiles/r6_qmoe_int8c_kmajor_bench.log)
        self.kmajor = bool(kmajor)
        if self.kmajor:
            G, nsb = self.N // 16, self.K // 256
            self.q = self.q.view(self.E, G, nsb, -1).transpose(1, 2).contiguous().view(self.E, -1)
        self.rs = (torch.stack([p.rs for p in parts]).contiguous() if p0.kqt in (6, 9)
                   else torch.empty(0, 0, dtype=torch.float32, device=p0.q.device))
        self.dense = None

    @property
    def shape(self):
        return (self.E, self.N, self.K)

    def dequantize(self, out: torch.Tensor | None = None) -> torch.Tensor:
        out = out if out is not None else torch.empty(self.E, self.N, self.K, dtype=torch.bfloat16,
                                                      device=self.q.device)
        # the stacked experts [E][N/16][K/256][chunk] are one tiled [E N, K] matrix: one launch
        torch.ops.hipserve.gguf_dequant_tiled(out.view(self.E * self.N, self.K), self.q.view(-1),
                                              self.rs.view(-1) if self.rs.numel() else self.rs,
                                              self.kqt, self.E * self.N, self.K, 0, self.N, self.kmajor)
        return out

    @staticmethod
    def supported(kqt: int, N: int, K: int) -> bool:
        return kqt in QuantMoE.KERNEL_QTS and N % 16 == 0 and K % 256 == 0


_MOE_SCRATCH: dict = {}


def moe_dense(w: QuantMoE, slot: int) -> torch.Tensor:
    """bf16 [E, N, K] experts for a prefill-sized MoE: the resident shadow, or one of two
    per-device scratch buffers (w13 / w2 of the current layer) dequantised now."""
    if w.dense is not None:
        return w.dense
    key = (w.q.device, slot)
    buf = _MOE_SCRATCH.get(key)
    n = w.E * w.N * w.K
    if buf is None or buf.numel() < n:
        buf = _MOE_SCRATCH[key] = torch.empty(n, dtype=torch.bfloat16, device=w.q.device)
    return w.dequantize(buf[:n].view(w.E, w.N, w.K))


_MOE_PACKED_SCRATCH: dict = {}


def moe_packed_scratch(w: QuantMoE, slot: int, glu: bool) -> torch.Tensor:
    """[E, packed] bf16 experts in the packed prefill GEMM's layout (``pack_decode_weight``,
    gate/up-interleaved for w13), dequantised straight into it (one launch over all
    experts, gguf_mfma.hip dequant_tiled_kernel pack mode): the operand of the one-launch
    grouped expert GEMM (prefill_gemm_packed.hip kGroup), in a per-device scratch."""
    if w.dense is not None:
        raise ValueError("moe_packed_scratch: experts with a bf16 shadow take the shadow path")
    key = (w.q.device, slot)
    n = w.E * (-(-w.N // 128) * 128) * w.K
    buf = _MOE_PACKED_SCRATCH.get(key)
    if buf is None or buf.numel() < n:
        buf = _MOE_PACKED_SCRATCH[key] = torch.empty(n, dtype=torch.bfloat16, device=w.q.device)
    out = buf[:n].view(w.E, n // w.E)
    torch.ops.hipserve.gguf_dequant_tiled(out.view(-1), w.q.view(-1), w.rs.view(-1) if w.rs.numel() else w.rs,
                                          w.kqt, w.E * w.N, w.K, 2 if glu else 1, w.N, w.kmajor)
    return out


def make_moe_shadows(moes, device, reserve_bytes: int) -> int:
    """bf16 shadows of quantised experts for prefill while ``reserve_bytes`` stay free."""
    import os

    if os.environ.get("HIPSERVE_QUANT_SHADOW", "1") == "0" or torch.device(device).type != "cuda":
        return 0
    added = 0
    for w in moes:
        need = w.E * w.N * w.K * 2
        free, _ = torch.cuda.mem_get_info(device)
        if w.dense is None and free - need >= reserve_bytes:
            w.dense = w.dequantize()
            added += need
    return added
