"""Quantised (GGUF) weights on the GPU and the matmul that consumes them.

``QuantWeight`` repacks GGUF blocks once at load into the layouts
``csrc/kernels/gguf.hip`` reads with aligned 16-byte loads (K-quants stay in their
native super-blocks, Q6_K is padded to 224 B, Q8_0/Q4_0/Q4_1 become
structure-of-arrays) and keeps merged projections (q|k|v, gate|up) as parts that
may use different formats (Q4_K_M puts attn_v/ffn_down in Q6_K).

``quant_linear(x, w)``: decode batches (M <= 64) run the fused dequant-in-register
MFMA GEMM; larger M (prefill) dequantises one part at a time into a reusable bf16
scratch and runs hipBLASLt.
"""
from __future__ import annotations

import numpy as np
import torch

from ..weights import gguf as G

KERNEL_QT = {G.Q4_0: 0, G.Q4_1: 1, G.Q8_0: 2, G.Q4_K: 3, G.Q5_K: 4, G.Q6_K: 5}
MAX_FUSED_M = 64


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


class QuantPart:
    def __init__(self, qtype, N, K, q, d, m, row_bytes):
        self.qtype, self.N, self.K = qtype, N, K
        self.kqt = KERNEL_QT[qtype]
        self.q, self.d, self.m, self.row_bytes = q, d, m, row_bytes

    @property
    def nbytes(self):
        return self.q.numel() + 2 * (self.d.numel() + self.m.numel())


class QuantWeight:
    def __init__(self, parts: list[QuantPart]):
        self.parts = parts
        self.N = sum(p.N for p in parts)
        self.K = parts[0].K
        assert all(p.K == self.K for p in parts)

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
            q, d, m, rb = repack(gf.raw(n), t.type, N, K)
            to = lambda a, dt: torch.from_numpy(np.array(a, copy=True, order='C')).view(dt).to(device)  # noqa: E731
            parts.append(QuantPart(t.type, N, K, to(q, torch.uint8), to(d, torch.int16),
                                   to(m, torch.int16), rb))
        return cls(parts)

    @classmethod
    def from_raw(cls, raws: list, device):
        """[(qtype, N, K, raw ggml bytes)] -> QuantWeight on ``device``."""
        parts = []
        for qtype, N, K, raw in raws:
            q, d, m, rb = repack(raw, qtype, N, K)
            to = lambda a, dt: torch.from_numpy(np.array(a, copy=True, order='C')).view(dt).to(device)  # noqa: E731
            parts.append(QuantPart(qtype, N, K, to(q, torch.uint8), to(d, torch.int16), to(m, torch.int16), rb))
        return cls(parts)

    @classmethod
    def from_float(cls, w: np.ndarray | list, qtype: int, device):
        """Quantise float matrices (tests / synthetic benchmarks)."""
        mats = w if isinstance(w, list) else [w]
        parts = []
        for mat in mats:
            mat = np.asarray(mat, np.float32)
            N, K = mat.shape
            q, d, m, rb = repack(G.quantize(mat, qtype), qtype, N, K)
            to = lambda a, dt: torch.from_numpy(np.array(a, copy=True, order='C')).view(dt).to(device)  # noqa: E731
            parts.append(QuantPart(qtype, N, K, to(q, torch.uint8), to(d, torch.int16), to(m, torch.int16), rb))
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


def dequantize(w: QuantWeight) -> torch.Tensor:
    outs = []
    for p in w.parts:
        o = torch.empty(p.N, p.K, dtype=torch.bfloat16, device=p.q.device)
        torch.ops.hipserve.gguf_dequant(o, p.q, p.d, p.m, p.kqt, p.row_bytes, p.N, p.K)
        outs.append(o)
    return torch.cat(outs, 0) if len(outs) > 1 else outs[0]


def _splits(N: int, K: int) -> int:
    """K slices for the decode dequant-GEMM: ~512 (64-row tile, K slice) workgroups."""
    wgs = (N + 63) // 64
    nsb = K // 256
    return max(1, min(nsb, -(-512 // wgs)))


def quant_linear(x: torch.Tensor, w: QuantWeight) -> torch.Tensor:
    M = x.shape[0]
    out = torch.empty(M, w.N, dtype=torch.bfloat16, device=x.device)
    if M == 0:
        return out
    if M <= MAX_FUSED_M:
        off = 0
        for p in w.parts:
            sp = _splits(p.N, p.K)
            ws = torch.empty(sp, M, p.N, dtype=torch.float32, device=x.device) if sp > 1 else \
                torch.empty(0, dtype=torch.float32, device=x.device)
            torch.ops.hipserve.gguf_gemm(out[:, off:off + p.N], x, p.q, p.d, p.m, p.kqt, p.row_bytes,
                                         p.N, p.K, ws, sp)
            off += p.N
        return out
    off = 0
    for p in w.parts:
        buf = _dequant_scratch(x.device, p.N * p.K)[: p.N * p.K].view(p.N, p.K)
        torch.ops.hipserve.gguf_dequant(buf, p.q, p.d, p.m, p.kqt, p.row_bytes, p.N, p.K)
        out[:, off:off + p.N] = torch.nn.functional.linear(x, buf)
        off += p.N
    return out
