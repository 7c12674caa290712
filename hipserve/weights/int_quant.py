"""Integer weight-only checkpoints (AWQ / GPTQ-style group quantisation), dequantised
to the compute dtype at load.

The reference's HF chart serves ``cpatonn/Qwen3-VL-30B-A3B-Instruct-AWQ-8bit``
(vllm-models/helm-chart/values.yaml:8-12): an llm-compressor export in the
compressed-tensors ``pack-quantized`` format. Two on-disk layouts are read:

* compressed-tensors ``pack-quantized`` (``quant_method: compressed-tensors``):
  ``<name>.weight_packed`` int32 [N, ceil(K / (32 / b))] — b-bit values stored with
  an offset of 2^(b-1) (signed -> unsigned), packed lowest bits first along K;
  ``<name>.weight_scale`` [N, K / group] (or [N, 1] per channel);
  optional ``<name>.weight_zero_point`` (asymmetric; signed, packed the same way
  along N, or unpacked [N, K / group]); optional ``<name>.weight_shape`` = (N, K).
  w = (q - zp) * scale.
* AutoAWQ ``gemm`` (``quant_method: awq``, 4-bit): ``<name>.qweight`` int32
  [K, N / 8], ``<name>.qzeros`` int32 [K / group, N / 8], ``<name>.scales``
  [K / group, N]; eight nibbles per int32 in AWQ's interleaved column order
  (0, 2, 4, 6, 1, 3, 5, 7). w^T = (q - z) * s.

On the GPU, 8-bit pack-quantized dense projections are NOT dequantised: the loader
(safetensors_loader.py ``int8_part``) keeps the bytes, group scales and zero points
and the v2 quantised decode GEMM (csrc/kernels/gguf_mfma.hip, INT8 format) dequantises
in registers — half the bf16 bytes per decode step. 4-bit layouts, AutoAWQ and MoE
expert weights are dequantised here to bf16 at load (288 GB of HBM holds a 30B-A3B
model in bf16 several times over).
"""
from __future__ import annotations

import torch

# nibble k of an AWQ int32 holds column AWQ_ORDER[k] of its 8-column group
AWQ_ORDER = (0, 2, 4, 6, 1, 3, 5, 7)


def _unpack_rows(packed: torch.Tensor, bits: int, n: int) -> torch.Tensor:
    """int32 [R, C] -> int32 [R, n] of unsigned b-bit values, lowest bits first."""
    pf = 32 // bits
    p = packed.to(torch.int64) & 0xFFFFFFFF
    shifts = torch.arange(pf, dtype=torch.int64) * bits
    v = (p.unsqueeze(-1) >> shifts) & ((1 << bits) - 1)
    return v.reshape(p.shape[0], -1)[:, :n].to(torch.int32)


def pack_rows(values: torch.Tensor, bits: int) -> torch.Tensor:
    """Inverse of :func:`_unpack_rows` (unsigned values [R, n] -> int32 [R, ceil(n/pf)])."""
    pf = 32 // bits
    R, n = values.shape
    pad = (-n) % pf
    v = torch.nn.functional.pad(values.to(torch.int64), (0, pad)).reshape(R, -1, pf)
    shifts = torch.arange(pf, dtype=torch.int64) * bits
    w = (v << shifts).sum(-1)
    return torch.where(w >= 1 << 31, w - (1 << 32), w).to(torch.int32)


def dequant_pack_quantized(packed, scale, zero_point=None, shape=None, bits=None) -> torch.Tensor:
    """compressed-tensors pack-quantized -> fp32 [N, K]."""
    N = packed.shape[0]
    if shape is not None:
        N, K = (int(x) for x in shape.reshape(-1).tolist())
    elif bits is not None:
        K = packed.shape[1] * (32 // bits)
    else:
        raise ValueError("pack-quantized tensor needs weight_shape or num_bits")
    if bits is None:  # weight_shape present: the packing factor gives the width
        pf = -(-K // packed.shape[1])
        bits = 32 // pf
    off = 1 << (bits - 1)
    q = (_unpack_rows(packed, bits, K) - off).float()
    scale = scale.float()
    if scale.dim() == 1:
        scale = scale.reshape(-1, 1)
    groups = scale.shape[1]
    g = -(-K // groups)
    if zero_point is not None:
        zp = zero_point
        if zp.dtype == torch.int32 and zp.shape[0] != N:  # packed along N
            zp = (_unpack_rows(zp.t().contiguous(), bits, N) - off).t()
        zp = zp.float().reshape(N, -1)
        q = q - zp.repeat_interleave(g, 1)[:, :K]
    return q * scale.repeat_interleave(g, 1)[:, :K]


def pack_pack_quantized(q: torch.Tensor, bits: int) -> torch.Tensor:
    """Signed b-bit integers [N, K] -> compressed-tensors ``weight_packed``."""
    return pack_rows(q.to(torch.int64) + (1 << (bits - 1)), bits)


def _awq_unpack(t: torch.Tensor) -> torch.Tensor:
    """AutoAWQ int32 [R, C] -> int32 [R, 8C] in natural column order."""
    v = _unpack_rows(t, 4, t.shape[1] * 8).reshape(t.shape[0], -1, 8)
    inv = [AWQ_ORDER.index(j) for j in range(8)]
    return v[:, :, inv].reshape(t.shape[0], -1)


def awq_pack(v: torch.Tensor) -> torch.Tensor:
    """Natural-order unsigned 4-bit [R, 8C] -> AutoAWQ int32 [R, C]."""
    R = v.shape[0]
    g = v.reshape(R, -1, 8)[:, :, list(AWQ_ORDER)].reshape(R, -1)
    return pack_rows(g, 4)


def dequant_awq(qweight, qzeros, scales) -> torch.Tensor:
    """AutoAWQ gemm -> fp32 [N, K] (the HF Linear layout)."""
    q = _awq_unpack(qweight).float()  # [K, N]
    z = _awq_unpack(qzeros).float()  # [K/g, N]
    s = scales.float()
    g = q.shape[0] // s.shape[0]
    return ((q - z.repeat_interleave(g, 0)) * s.repeat_interleave(g, 0)).t().contiguous()
