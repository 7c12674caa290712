"""GGUF (llama.cpp model file) support for the GGUF tier.

The reference's GGUF tier runs ``llama-server --model <file.gguf> --alias <name>``
(ramalama-models/helm-chart/templates/model-deployments.yaml:26-35) on files
like TinyLlama Q8_0 / Phi-3-mini q4 (ramalama-models/README.md:103-106). This
module is hipserve's in-house replacement for llama.cpp's loader (no ``gguf``
Python package is available):

* ``GGUFFile``    — zero-copy parser (``numpy.memmap``) of header, metadata and
  tensor infos (GGUF v2/v3), ``model_config()`` from ``llama.*`` metadata;
* block codecs    — numpy reference dequantisers (and quantisers, used to write
  synthetic test/benchmark files) for F32/F16/BF16/Q8_0/Q4_0/Q4_1/Q5_0/Q5_1/
  Q4_K/Q5_K/Q6_K, bit-exact with ggml's block layouts;
* ``GGUFTokenizer`` — SentencePiece-BPE (``llama``) and byte-level BPE (``gpt2``,
  Llama-3) tokenizers built from the embedded vocab;
* ``load_gguf_weights`` — maps ``blk.N.*`` tensors onto the hipserve model; the
  quantised matrices stay quantised on the GPU (``QuantWeight``) and are consumed
  by the gfx950 dequant-GEMV / dequant-GEMM kernels.
GGUF Q/K projection rows are pre-permuted for interleaved rotary pairs, so the
model runs RoPE in "interleaved" mode (rope_mode = 1).
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

import numpy as np

GGUF_MAGIC = b"GGUF"

# ggml tensor types (ggml.h)
F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1 = 0, 1, 2, 3, 6, 7, 8, 9
Q2_K, Q3_K, Q4_K, Q5_K, Q6_K, Q8_K = 10, 11, 12, 13, 14, 15
BF16 = 30
TYPE_NAMES = {F32: "F32", F16: "F16", Q4_0: "Q4_0", Q4_1: "Q4_1", Q5_0: "Q5_0", Q5_1: "Q5_1",
              Q8_0: "Q8_0", Q8_1: "Q8_1", Q2_K: "Q2_K", Q3_K: "Q3_K", Q4_K: "Q4_K", Q5_K: "Q5_K",
              Q6_K: "Q6_K", Q8_K: "Q8_K", BF16: "BF16"}
# (block elements, bytes per block)
BLOCK = {F32: (1, 4), F16: (1, 2), BF16: (1, 2), Q4_0: (32, 18), Q4_1: (32, 20), Q5_0: (32, 22),
         Q5_1: (32, 24), Q8_0: (32, 34), Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210)}

# metadata value types
_U8, _I8, _U16, _I16, _U32, _I32, _F32, _BOOL, _STR, _ARR, _U64, _I64, _F64 = range(13)
_SCALAR = {_U8: "<B", _I8: "<b", _U16: "<H", _I16: "<h", _U32: "<I", _I32: "<i", _F32: "<f",
           _BOOL: "<?", _U64: "<Q", _I64: "<q", _F64: "<d"}
_NP = {_U8: np.uint8, _I8: np.int8, _U16: np.uint16, _I16: np.int16, _U32: np.uint32,
       _I32: np.int32, _F32: np.float32, _BOOL: np.bool_, _U64: np.uint64, _I64: np.int64,
       _F64: np.float64}


@dataclass
class TensorInfo:
    name: str
    shape: tuple          # ggml order: ne[0] = innermost (row length)
    type: int
    offset: int           # relative to the data section

    @property
    def n_elements(self):
        n = 1
        for d in self.shape:
            n *= d
        return n

    @property
    def nbytes(self):
        be, bb = BLOCK[self.type]
        return self.n_elements // be * bb

    @property
    def rows_cols(self):
        """(rows, row_length) of the row-major matrix."""
        cols = self.shape[0]
        return self.n_elements // cols, cols


class GGUFFile:
    def __init__(self, path: str):
        self.path = path
        self.mm = np.memmap(path, dtype=np.uint8, mode="r")
        self.metadata: dict = {}
        self.tensors: dict[str, TensorInfo] = {}
        self._parse()

    # -------------------------------------------------------------- parsing
    def _parse(self):
        buf = self.mm
        if bytes(buf[:4]) != GGUF_MAGIC:
            raise ValueError(f"{self.path}: not a GGUF file")
        self.version = struct.unpack_from("<I", buf, 4)[0]
        if self.version not in (2, 3):
            raise ValueError(f"unsupported GGUF version {self.version}")
        n_tensors, n_kv = struct.unpack_from("<QQ", buf, 8)
        pos = 24
        for _ in range(n_kv):
            key, pos = self._str(pos)
            vtype = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
            val, pos = self._value(vtype, pos)
            self.metadata[key] = val
        for _ in range(n_tensors):
            name, pos = self._str(pos)
            nd = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
            shape = struct.unpack_from(f"<{nd}Q", buf, pos)
            pos += 8 * nd
            ttype, off = struct.unpack_from("<IQ", buf, pos)
            pos += 12
            self.tensors[name] = TensorInfo(name, tuple(int(x) for x in shape), ttype, off)
        align = int(self.metadata.get("general.alignment", 32))
        self.data_offset = (pos + align - 1) // align * align

    def _str(self, pos):
        n = struct.unpack_from("<Q", self.mm, pos)[0]
        pos += 8
        return bytes(self.mm[pos:pos + n]).decode("utf-8", errors="replace"), pos + n

    def _value(self, vtype, pos):
        if vtype in _SCALAR:
            fmt = _SCALAR[vtype]
            return struct.unpack_from(fmt, self.mm, pos)[0], pos + struct.calcsize(fmt)
        if vtype == _STR:
            return self._str(pos)
        if vtype == _ARR:
            et, n = struct.unpack_from("<IQ", self.mm, pos)
            pos += 12
            if et in _NP:
                dt = np.dtype(_NP[et])
                arr = np.frombuffer(self.mm, dtype=dt, count=n, offset=pos).copy()
                return arr, pos + n * dt.itemsize
            out = []
            for _ in range(n):
                v, pos = self._value(et, pos)
                out.append(v)
            return out, pos
        raise ValueError(f"bad GGUF metadata type {vtype}")

    # -------------------------------------------------------------- access
    def raw(self, name: str) -> np.ndarray:
        """Raw bytes of a tensor (zero-copy view of the mmap)."""
        t = self.tensors[name]
        s = self.data_offset + t.offset
        return self.mm[s:s + t.nbytes]

    def tensor_f32(self, name: str) -> np.ndarray:
        t = self.tensors[name]
        rows, cols = t.rows_cols
        return dequantize(self.raw(name), t.type, t.n_elements).reshape(rows, cols) \
            if len(t.shape) > 1 else dequantize(self.raw(name), t.type, t.n_elements)

    def arch(self) -> str:
        return self.metadata.get("general.architecture", "llama")

    def model_config(self, name: str | None = None):
        from ..config import ModelConfig

        md, a = self.metadata, self.arch()
        g = lambda k, d=None: md.get(f"{a}.{k}", d)  # noqa: E731
        nh = int(g("attention.head_count"))
        H = int(g("embedding_length"))
        tok = md.get("tokenizer.ggml.tokens")
        V = len(tok) if tok is not None else self.tensors["token_embd.weight"].shape[1]
        head_dim = int(g("attention.key_length", H // nh))
        eos = md.get("tokenizer.ggml.eos_token_id", 2)
        eos_ids = {int(eos)}
        if md.get("tokenizer.ggml.eot_token_id") is not None:
            eos_ids.add(int(md["tokenizer.ggml.eot_token_id"]))
        n_exp = int(g("expert_count", 0) or 0)
        if a not in GGUF_ARCHS:
            raise NotImplementedError(f"GGUF architecture {a!r} (supported: {', '.join(GGUF_ARCHS)})")
        if int(g("rope.dimension_count", head_dim) or head_dim) != head_dim:
            raise NotImplementedError("partial rotary embeddings are not supported")
        fam = {"llama": "mixtral" if n_exp else "llama"}.get(a, a)
        return ModelConfig(
            name=name or md.get("general.name", os.path.basename(self.path)),
            architecture="mixtral" if n_exp else "llama", family=fam,
            hidden_size=H, num_layers=int(g("block_count")), num_heads=nh,
            num_kv_heads=int(g("attention.head_count_kv", nh)), head_dim=head_dim,
            intermediate_size=int(g("feed_forward_length")), vocab_size=V,
            rms_norm_eps=float(g("attention.layer_norm_rms_epsilon", 1e-5)),
            # llama.cpp permutes llama q/k rows for interleaved RoPE; phi3 / qwen run NeoX RoPE
            rope_theta=float(g("rope.freq_base", 10000.0)), rope_mode=1 if a == "llama" else 0,
            max_position_embeddings=int(g("context_length", 4096)),
            tie_word_embeddings="output.weight" not in self.tensors,
            num_experts=n_exp, num_experts_per_tok=int(g("expert_used_count", 0) or 0),
            qkv_bias=a == "qwen2", qk_norm=a == "qwen3",
            bos_token_id=int(md.get("tokenizer.ggml.bos_token_id", 1)),
            eos_token_id=tuple(sorted(eos_ids)))


# ------------------------------------------------------------------ codecs
def _f16(b: np.ndarray) -> np.ndarray:
    return b.copy().view(np.float16).astype(np.float32)


def _scale_min_k4(scales: np.ndarray):
    """[nb, 12] packed 6-bit scales/mins -> (sc[nb, 8], m[nb, 8])"""
    s = scales.astype(np.uint8)
    sc = np.empty((s.shape[0], 8), np.uint8)
    mn = np.empty((s.shape[0], 8), np.uint8)
    sc[:, :4] = s[:, 0:4] & 63
    mn[:, :4] = s[:, 4:8] & 63
    sc[:, 4:] = (s[:, 8:12] & 0xF) | ((s[:, 0:4] >> 6) << 4)
    mn[:, 4:] = (s[:, 8:12] >> 4) | ((s[:, 4:8] >> 6) << 4)
    return sc.astype(np.float32), mn.astype(np.float32)


def dequantize(raw: np.ndarray, qtype: int, n: int) -> np.ndarray:
    raw = np.asarray(raw, dtype=np.uint8)
    if qtype == F32:
        return raw.view(np.float32)[:n].astype(np.float32)
    if qtype == F16:
        return raw.view(np.float16)[:n].astype(np.float32)
    if qtype == BF16:
        return (raw.view(np.uint16)[:n].astype(np.uint32) << 16).view(np.float32)
    be, bb = BLOCK[qtype]
    nb = n // be
    b = raw[: nb * bb].reshape(nb, bb)
    if qtype == Q8_0:
        d = _f16(b[:, 0:2])
        q = b[:, 2:34].view(np.int8).astype(np.float32)
        return (d * q).reshape(-1)
    if qtype in (Q4_0, Q4_1):
        off = 2 if qtype == Q4_0 else 4
        d = _f16(b[:, 0:2])
        qs = b[:, off:off + 16]
        lo, hi = (qs & 0xF).astype(np.float32), (qs >> 4).astype(np.float32)
        q = np.concatenate([lo, hi], axis=1)
        if qtype == Q4_0:
            return (d * (q - 8)).reshape(-1)
        return (d * q + _f16(b[:, 2:4])).reshape(-1)
    if qtype in (Q5_0, Q5_1):
        off = 2 if qtype == Q5_0 else 4
        d = _f16(b[:, 0:2])
        qh = b[:, off:off + 4].copy().view(np.uint32)[:, 0]
        qs = b[:, off + 4:off + 20]
        bits = (qh[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1
        lo = (qs & 0xF) | (bits[:, :16] << 4).astype(np.uint8)
        hi = (qs >> 4) | (bits[:, 16:] << 4).astype(np.uint8)
        q = np.concatenate([lo, hi], axis=1).astype(np.float32)
        if qtype == Q5_0:
            return (d * (q - 16)).reshape(-1)
        return (d * q + _f16(b[:, 2:4])).reshape(-1)
    if qtype == Q4_K:
        d, dmin = _f16(b[:, 0:2]), _f16(b[:, 2:4])
        sc, mn = _scale_min_k4(b[:, 4:16])
        qs = b[:, 16:144].reshape(nb, 4, 32)
        out = np.empty((nb, 8, 32), np.float32)
        out[:, 0::2] = (qs & 0xF).astype(np.float32)
        out[:, 1::2] = (qs >> 4).astype(np.float32)
        out = (d[:, :, None] * sc[:, :, None]) * out - (dmin[:, :, None] * mn[:, :, None])
        return out.reshape(-1)
    if qtype == Q5_K:
        d, dmin = _f16(b[:, 0:2]), _f16(b[:, 2:4])
        sc, mn = _scale_min_k4(b[:, 4:16])
        qh = b[:, 16:48]                     # [nb, 32]
        qs = b[:, 48:176].reshape(nb, 4, 32)
        out = np.empty((nb, 8, 32), np.float32)
        for j in range(4):
            h_lo = ((qh >> (2 * j)) & 1).astype(np.uint8) << 4
            h_hi = ((qh >> (2 * j + 1)) & 1).astype(np.uint8) << 4
            out[:, 2 * j] = ((qs[:, j] & 0xF) | h_lo).astype(np.float32)
            out[:, 2 * j + 1] = ((qs[:, j] >> 4) | h_hi).astype(np.float32)
        out = (d[:, :, None] * sc[:, :, None]) * out - (dmin[:, :, None] * mn[:, :, None])
        return out.reshape(-1)
    if qtype == Q6_K:
        ql = b[:, 0:128].reshape(nb, 2, 64)
        qh = b[:, 128:192].reshape(nb, 2, 32)
        scl = b[:, 192:208].view(np.int8).astype(np.float32).reshape(nb, 2, 8)
        d = _f16(b[:, 208:210])
        out = np.empty((nb, 2, 4, 32), np.float32)
        for h in range(2):
            l0, l1, hh = ql[:, h, :32], ql[:, h, 32:], qh[:, h]
            q1 = ((l0 & 0xF) | ((hh >> 0) & 3) << 4).astype(np.int32) - 32
            q2 = ((l1 & 0xF) | ((hh >> 2) & 3) << 4).astype(np.int32) - 32
            q3 = ((l0 >> 4) | ((hh >> 4) & 3) << 4).astype(np.int32) - 32
            q4 = ((l1 >> 4) | ((hh >> 6) & 3) << 4).astype(np.int32) - 32
            for qi, q in enumerate((q1, q2, q3, q4)):
                # scale index: is = l/16 (+2*qi) -> lanes 0..15 use sc[2qi], 16..31 sc[2qi+1]
                s = np.repeat(scl[:, h, 2 * qi:2 * qi + 2], 16, axis=1)
                out[:, h, qi] = d * s * q
        return out.reshape(-1)
    raise NotImplementedError(f"GGUF type {TYPE_NAMES.get(qtype, qtype)} not supported")


def _to_f16_bytes(x: np.ndarray) -> np.ndarray:
    return x.astype(np.float16).view(np.uint8).reshape(-1, 2)


def quantize(x: np.ndarray, qtype: int) -> np.ndarray:
    """Reference quantiser (round-to-nearest, ggml block layouts) -> raw bytes."""
    x = np.asarray(x, np.float32).reshape(-1)
    if qtype == F32:
        return x.view(np.uint8).copy()
    if qtype == F16:
        return x.astype(np.float16).view(np.uint8).copy()
    if qtype == BF16:
        u = x.view(np.uint32)
        return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16).view(np.uint8).copy()
    be, bb = BLOCK[qtype]
    nb = x.size // be
    xb = x[: nb * be].reshape(nb, be)
    out = np.zeros((nb, bb), np.uint8)
    if qtype == Q8_0:
        amax = np.abs(xb).max(1)
        d = (amax / 127.0).astype(np.float16).astype(np.float32)
        inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0)
        q = np.clip(np.round(xb * inv[:, None]), -127, 127).astype(np.int8)
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:34] = q.view(np.uint8)
        return out.reshape(-1)
    if qtype == Q4_0:
        idx = np.abs(xb).argmax(1)
        mx = xb[np.arange(nb), idx]
        d = (mx / -8.0).astype(np.float16).astype(np.float32)
        inv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0)
        q = np.clip(np.floor(xb * inv[:, None] + 8.5), 0, 15).astype(np.uint8)
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:18] = q[:, :16] | (q[:, 16:] << 4)
        return out.reshape(-1)
    if qtype in (Q4_K, Q5_K):
        nbits = 4 if qtype == Q4_K else 5
        qmax = (1 << nbits) - 1
        sub = xb.reshape(nb, 8, 32)
        mn = np.minimum(sub.min(2), 0)
        mx = sub.max(2)
        scale = np.maximum((mx - mn) / qmax, 1e-12)
        d = (scale.max(1) / 63).astype(np.float16).astype(np.float32)
        dmin = ((-mn).max(1) / 63).astype(np.float16).astype(np.float32)
        ls = np.clip(np.round(scale / np.where(d > 0, d, 1)[:, None]), 0, 63).astype(np.uint8)
        lm = np.clip(np.round(-mn / np.where(dmin > 0, dmin, 1)[:, None]), 0, 63).astype(np.uint8)
        eff_s = d[:, None] * ls
        eff_m = dmin[:, None] * lm
        q = np.clip(np.round((sub + eff_m[:, :, None]) / np.where(eff_s > 0, eff_s, 1)[:, :, None]),
                    0, qmax).astype(np.uint8)
        sc = np.zeros((nb, 12), np.uint8)
        sc[:, 0:4] = ls[:, :4] | ((ls[:, 4:] >> 4) << 6)
        sc[:, 4:8] = lm[:, :4] | ((lm[:, 4:] >> 4) << 6)
        sc[:, 8:12] = (ls[:, 4:] & 0xF) | ((lm[:, 4:] & 0xF) << 4)
        out[:, 0:2] = _to_f16_bytes(d)
        out[:, 2:4] = _to_f16_bytes(dmin)
        out[:, 4:16] = sc
        if qtype == Q4_K:
            qq = q.reshape(nb, 4, 2, 32)
            out[:, 16:144] = (qq[:, :, 0] | (qq[:, :, 1] << 4)).reshape(nb, 128)
        else:
            qq = q.reshape(nb, 4, 2, 32)
            lo = qq & 0xF
            out[:, 48:176] = (lo[:, :, 0] | (lo[:, :, 1] << 4)).reshape(nb, 128)
            qh = np.zeros((nb, 32), np.uint8)
            for j in range(4):
                qh |= ((qq[:, j, 0] >> 4) & 1) << (2 * j)
                qh |= ((qq[:, j, 1] >> 4) & 1) << (2 * j + 1)
            out[:, 16:48] = qh
        return out.reshape(-1)
    if qtype == Q6_K:
        sub = xb.reshape(nb, 16, 16)
        amax = np.abs(sub).max(2)
        s = amax / 31.0
        d = (s.max(1) / 127).astype(np.float16).astype(np.float32)
        ls = np.clip(np.round(s / np.where(d > 0, d, 1)[:, None]), -128, 127).astype(np.int8)
        eff = d[:, None] * ls.astype(np.float32)
        q = (np.clip(np.round(sub / np.where(eff != 0, eff, 1)[:, :, None]), -32, 31) + 32).astype(np.uint8)
        q = q.reshape(nb, 2, 4, 32)  # [half, quarter, l]
        ql = np.zeros((nb, 2, 64), np.uint8)
        qh = np.zeros((nb, 2, 32), np.uint8)
        ql[:, :, :32] = (q[:, :, 0] & 0xF) | ((q[:, :, 2] & 0xF) << 4)
        ql[:, :, 32:] = (q[:, :, 1] & 0xF) | ((q[:, :, 3] & 0xF) << 4)
        qh[:] = (q[:, :, 0] >> 4) | ((q[:, :, 1] >> 4) << 2) | ((q[:, :, 2] >> 4) << 4) | ((q[:, :, 3] >> 4) << 6)
        out[:, 0:128] = ql.reshape(nb, 128)
        out[:, 128:192] = qh.reshape(nb, 64)
        out[:, 192:208] = ls.view(np.uint8)
        out[:, 208:210] = _to_f16_bytes(d)
        return out.reshape(-1)
    raise NotImplementedError(f"quantize to {TYPE_NAMES.get(qtype, qtype)}")


# ------------------------------------------------------------------ writer
def _w_str(f, s: str):
    b = s.encode()
    f.write(struct.pack("<Q", len(b)))
    f.write(b)


def _w_val(f, v):
    if isinstance(v, bool):
        f.write(struct.pack("<I?", _BOOL, v))
    elif isinstance(v, int):
        f.write(struct.pack("<Iq" if v < 0 else "<IQ", _I64 if v < 0 else _U64, v)) if abs(v) >= 2**31 \
            else f.write(struct.pack("<Ii", _I32, v))
    elif isinstance(v, float):
        f.write(struct.pack("<If", _F32, v))
    elif isinstance(v, str):
        f.write(struct.pack("<I", _STR))
        _w_str(f, v)
    elif isinstance(v, (list, tuple, np.ndarray)):
        f.write(struct.pack("<I", _ARR))
        items = list(v)
        if items and isinstance(items[0], str):
            f.write(struct.pack("<IQ", _STR, len(items)))
            for s in items:
                _w_str(f, s)
        elif items and isinstance(items[0], (float, np.floating)):
            f.write(struct.pack("<IQ", _F32, len(items)))
            f.write(np.asarray(items, np.float32).tobytes())
        else:
            f.write(struct.pack("<IQ", _I32, len(items)))
            f.write(np.asarray(items, np.int32).tobytes())
    else:
        raise TypeError(type(v))


def write_gguf(path: str, metadata: dict, tensors: list[tuple[str, np.ndarray, int]],
               alignment: int = 32):
    """tensors: (name, float32 array [rows, cols] or [n], ggml type)."""
    blobs = []
    for name, arr, qt in tensors:
        a = np.asarray(arr, np.float32)
        shape = tuple(reversed(a.shape))  # ggml ne order
        blobs.append((name, shape, qt, quantize(a, qt).tobytes()))
    with open(path, "wb") as f:
        f.write(GGUF_MAGIC)
        f.write(struct.pack("<IQQ", 3, len(blobs), len(metadata) + 1))
        _w_str(f, "general.alignment")
        f.write(struct.pack("<II", _U32, alignment))
        for k, v in metadata.items():
            _w_str(f, k)
            _w_val(f, v)
        off = 0
        offsets = []
        for name, shape, qt, data in blobs:
            _w_str(f, name)
            f.write(struct.pack("<I", len(shape)))
            f.write(struct.pack(f"<{len(shape)}Q", *shape))
            f.write(struct.pack("<IQ", qt, off))
            offsets.append(off)
            off += (len(data) + alignment - 1) // alignment * alignment
        pad = (-f.tell()) % alignment
        f.write(b"\0" * pad)
        for (name, shape, qt, data), o in zip(blobs, offsets):
            f.write(data)
            f.write(b"\0" * ((-len(data)) % alignment))


# ------------------------------------------------------------------ tokenizer
class GGUFTokenizer:
    """Tokenizer from GGUF metadata: ``llama`` (SentencePiece BPE with scores and
    <0xXX> byte fallback) or ``gpt2`` (byte-level BPE with merges, Llama-3)."""

    def __init__(self, gf: GGUFFile):
        from ..tokenizer import BaseTokenizer, _DEFAULT_CHAT_TEMPLATE

        md = gf.metadata
        self.kind = md.get("tokenizer.ggml.model", "llama")
        self.tokens = list(md["tokenizer.ggml.tokens"])
        self.vocab_size = len(self.tokens)
        self.scores = md.get("tokenizer.ggml.scores")
        self.types = md.get("tokenizer.ggml.token_type")
        self.id = {t: i for i, t in enumerate(self.tokens)}
        self.bos_token_id = int(md.get("tokenizer.ggml.bos_token_id", 1))
        eos = {int(md.get("tokenizer.ggml.eos_token_id", 2))}
        if md.get("tokenizer.ggml.eot_token_id") is not None:
            eos.add(int(md["tokenizer.ggml.eot_token_id"]))
        self.eos_token_ids = tuple(sorted(eos))
        self.add_bos = bool(md.get("tokenizer.ggml.add_bos_token", True))
        self.bos_token = self.tokens[self.bos_token_id] if self.bos_token_id < len(self.tokens) else ""
        self.eos_token = self.tokens[min(self.eos_token_ids)] if self.eos_token_ids else ""
        self.chat_template = md.get("tokenizer.chat_template") or _DEFAULT_CHAT_TEMPLATE
        self.special = set()
        if self.types is not None:
            self.special = {i for i, t in enumerate(self.types) if int(t) in (3, 4)}  # control/user-defined
        self._base = BaseTokenizer
        self.model_config_override = None
        if self.kind == "gpt2":
            merges = md.get("tokenizer.ggml.merges") or []
            self.ranks = {tuple(m.split(" ", 1)): i for i, m in enumerate(merges)}
            bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
                list(range(ord("®"), ord("ÿ") + 1))
            cs = bs[:]
            n = 0
            for b in range(256):
                if b not in bs:
                    bs.append(b)
                    cs.append(256 + n)
                    n += 1
            self.b2u = {b: chr(c) for b, c in zip(bs, cs)}
            self.u2b = {v: k for k, v in self.b2u.items()}
            import regex

            self.pat = regex.compile(
                r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+")
        self._special_sorted = sorted((self.tokens[i] for i in self.special if self.tokens[i]),
                                      key=len, reverse=True)

    # -- shared helpers from BaseTokenizer
    def apply_chat_template(self, messages, add_generation_prompt=True):
        from ..tokenizer import render_chat

        return render_chat(self.chat_template, messages, self.bos_token, self.eos_token, add_generation_prompt)

    def encode_chat(self, messages, add_generation_prompt=True):
        return self.encode(self.apply_chat_template(messages, add_generation_prompt), add_special_tokens=False,
                           parse_special=True)

    def _split_special(self, text):
        if not self._special_sorted:
            return [(False, text)]
        out, i, start = [], 0, 0
        while i < len(text):
            for s in self._special_sorted:
                if text.startswith(s, i):
                    if start < i:
                        out.append((False, text[start:i]))
                    out.append((True, s))
                    i += len(s)
                    start = i
                    break
            else:
                i += 1
        if start < len(text):
            out.append((False, text[start:]))
        return out

    def encode(self, text: str, add_special_tokens: bool = True, parse_special: bool = True) -> list[int]:
        ids = []
        if add_special_tokens and self.add_bos:
            ids.append(self.bos_token_id)
        parts = self._split_special(text) if parse_special else [(False, text)]
        first = True
        for is_sp, piece in parts:
            if is_sp:
                ids.append(self.id[piece])
            elif self.kind == "gpt2":
                ids += self._bpe_encode(piece)
            else:
                ids += self._spm_encode(piece, add_prefix=first)
            first = False
        return ids

    def _spm_encode(self, text: str, add_prefix: bool) -> list[int]:
        import heapq

        if not text:
            return []
        t = text.replace(" ", "▁")
        if add_prefix:
            t = "▁" + t
        syms = list(t)
        score = lambda s: float(self.scores[self.id[s]]) if s in self.id and self.scores is not None else 0.0  # noqa: E731
        # linked list over symbols; merge the highest-scoring adjacent pair first
        prev = list(range(-1, len(syms) - 1))
        nxt = list(range(1, len(syms) + 1))
        nxt[-1] = -1
        heap = []
        for i in range(len(syms) - 1):
            s = syms[i] + syms[i + 1]
            if s in self.id:
                heapq.heappush(heap, (-score(s), i, s))
        alive = [True] * len(syms)
        while heap:
            _, i, s = heapq.heappop(heap)
            j = nxt[i]
            if not alive[i] or j < 0 or not alive[j] or syms[i] + syms[j] != s:
                continue
            syms[i] = s
            alive[j] = False
            nxt[i] = nxt[j]
            if nxt[j] >= 0:
                prev[nxt[j]] = i
            if prev[i] >= 0:
                p = prev[i]
                ps = syms[p] + syms[i]
                if ps in self.id:
                    heapq.heappush(heap, (-score(ps), p, ps))
            if nxt[i] >= 0:
                ns = syms[i] + syms[nxt[i]]
                if ns in self.id:
                    heapq.heappush(heap, (-score(ns), i, ns))
        out = []
        i = 0
        while i >= 0 and i < len(syms):
            if alive[i]:
                s = syms[i]
                if s in self.id:
                    out.append(self.id[s])
                else:  # byte fallback
                    for b in s.encode("utf-8"):
                        out.append(self.id.get(f"<0x{b:02X}>", 0))
            i = nxt[i] if alive[i] else i + 1
        return out

    def _bpe_encode(self, text: str) -> list[int]:
        out = []
        for word in self.pat.findall(text):
            w = [self.b2u[b] for b in word.encode("utf-8")]
            while len(w) > 1:
                best, bi = None, -1
                for i in range(len(w) - 1):
                    r = self.ranks.get((w[i], w[i + 1]))
                    if r is not None and (best is None or r < best):
                        best, bi = r, i
                if best is None:
                    break
                w = w[:bi] + [w[bi] + w[bi + 1]] + w[bi + 2:]
            out += [self.id[x] for x in w if x in self.id]
        return out

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        if self.kind == "gpt2":
            bs = bytearray()
            for i in ids:
                i = int(i)
                if skip_special_tokens and i in self.special:
                    continue
                for ch in self.tokens[i]:
                    if ch in self.u2b:
                        bs.append(self.u2b[ch])
                    else:
                        bs += ch.encode()
            return bs.decode("utf-8", errors="replace")
        bs = bytearray()
        for i in ids:
            i = int(i)
            if i >= len(self.tokens) or (skip_special_tokens and i in self.special):
                continue
            t = self.tokens[i]
            if len(t) == 6 and t.startswith("<0x") and t.endswith(">"):
                bs.append(int(t[3:5], 16))
            else:
                bs += t.encode()
        return bs.decode("utf-8", errors="replace").replace("▁", " ")


# ------------------------------------------------------------------ loading
# llama.cpp architectures the GGUF tier serves (the reference's GGUF chart runs
# TinyLlama (llama) and Phi-3-mini (phi3): ramalama-models/helm-chart/values.yaml:3-19)
GGUF_ARCHS = ("llama", "phi3", "qwen2", "qwen3")


def gguf_name_map(layer: int) -> dict:
    p = f"blk.{layer}."
    return {"attn_norm": p + "attn_norm.weight", "q": p + "attn_q.weight", "k": p + "attn_k.weight",
            "v": p + "attn_v.weight", "o": p + "attn_output.weight", "ffn_norm": p + "ffn_norm.weight",
            "gate": p + "ffn_gate.weight", "up": p + "ffn_up.weight", "down": p + "ffn_down.weight"}


def load_gguf_weights(model, path: str):
    """Load a GGUF llama model. Matrices in quantised formats are kept quantised
    on the device (``QuantWeight``) for the fused dequant kernels; norms, F32/F16/
    BF16 matrices and the embedding table become bf16 tensors."""
    import torch

    from ..models.llama import LayerWeights
    from ..ops.quant import QuantWeight

    gf = GGUFFile(path)
    cfg, dev, dt = model.cfg, model.device, model.dtype
    if model.tp.world_size != 1:
        raise NotImplementedError("GGUF tier runs TP=1 (one device per pod, like llama-server)")

    def dense(name):
        t = gf.tensor_f32(name)
        return torch.from_numpy(np.ascontiguousarray(t)).to(device=dev, dtype=dt)

    def norm(name):
        return torch.from_numpy(gf.tensor_f32(name).astype(np.float32)).to(device=dev, dtype=dt)

    def matrix(*names):
        infos = [gf.tensors[n] for n in names]
        if all(i.type in (F32, F16, BF16) for i in infos) or dev.type != "cuda":
            return torch.cat([dense(n) for n in names], 0) if len(names) > 1 else dense(names[0])
        return QuantWeight.from_gguf(gf, names, dev)

    model.embed = dense("token_embd.weight")
    model.norm = norm("output_norm.weight")
    model.lm_head = matrix("output.weight") if "output.weight" in gf.tensors else model.embed
    model.layers = []
    for i in range(cfg.num_layers):
        n = gguf_name_map(i)
        p = f"blk.{i}."
        # phi3: fused attn_qkv [q; k; v] and ffn_up holding [gate; up] (no ffn_gate)
        qkv = matrix(p + "attn_qkv.weight") if p + "attn_qkv.weight" in gf.tensors else \
            matrix(n["q"], n["k"], n["v"])
        gu = matrix(n["gate"], n["up"]) if n["gate"] in gf.tensors else matrix(n["up"])
        lw = LayerWeights(ln1=norm(n["attn_norm"]), wqkv=qkv, wo=matrix(n["o"]), ln2=norm(n["ffn_norm"]),
                          wgu=gu, wd=matrix(n["down"]))
        if cfg.qkv_bias:  # qwen2
            lw.bqkv = torch.cat([dense(p + f"attn_{x}.bias") for x in ("q", "k", "v")]).contiguous()
        if cfg.qk_norm:  # qwen3
            lw.q_norm = torch.from_numpy(gf.tensor_f32(p + "attn_q_norm.weight").astype(np.float32)).to(dev)
            lw.k_norm = torch.from_numpy(gf.tensor_f32(p + "attn_k_norm.weight").astype(np.float32)).to(dev)
        model.layers.append(lw)
    from ..ops.quant import quant_linear

    model.quant_linear = quant_linear
    model.gguf = gf
    return gf


def write_synthetic_llama_gguf(path: str, cfg, qtype: int = Q8_0, seed: int = 0, std: float = 0.05,
                               vocab_tokens: list[str] | None = None, mixed_k: bool = False):
    """Write a random-weight llama GGUF (tests and GGUF-tier benchmarks; no
    network means no real checkpoints). ``mixed_k`` mimics Q4_K_M: attn_v and
    ffn_down in Q6_K, the rest in Q4_K."""
    rng = np.random.default_rng(seed)
    H, I, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    nq, nkv, V = cfg.num_heads, cfg.num_kv_heads, cfg.vocab_size

    def r(*s):
        return (rng.standard_normal(s) * std).astype(np.float32)

    toks = vocab_tokens or (["<unk>", "<s>", "</s>"] + [f"<0x{b:02X}>" for b in range(256)] +
                            [f"▁w{i}" for i in range(V - 259)])
    md = {"general.architecture": "llama", "general.name": cfg.name,
          "llama.context_length": cfg.max_position_embeddings, "llama.embedding_length": H,
          "llama.block_count": cfg.num_layers, "llama.feed_forward_length": I,
          "llama.attention.head_count": nq, "llama.attention.head_count_kv": nkv,
          "llama.rope.freq_base": float(cfg.rope_theta), "llama.rope.dimension_count": D,
          "llama.attention.layer_norm_rms_epsilon": float(cfg.rms_norm_eps),
          "tokenizer.ggml.model": "llama", "tokenizer.ggml.tokens": toks,
          "tokenizer.ggml.scores": [float(-i) for i in range(len(toks))],
          "tokenizer.ggml.token_type": [3 if i < 3 else (6 if 3 <= i < 259 else 1) for i in range(len(toks))],
          "tokenizer.ggml.bos_token_id": 1, "tokenizer.ggml.eos_token_id": 2}
    k4 = Q4_K if mixed_k else qtype
    k6 = Q6_K if mixed_k else qtype
    tensors = [("token_embd.weight", r(V, H), F16), ("output_norm.weight", 1 + r(H), F32),
               ("output.weight", r(V, H), k6)]
    for i in range(cfg.num_layers):
        n = gguf_name_map(i)
        tensors += [(n["attn_norm"], 1 + r(H), F32), (n["q"], r(nq * D, H), k4), (n["k"], r(nkv * D, H), k4),
                    (n["v"], r(nkv * D, H), k6), (n["o"], r(H, nq * D), k4), (n["ffn_norm"], 1 + r(H), F32),
                    (n["gate"], r(I, H), k4), (n["up"], r(I, H), k4), (n["down"], r(H, I), k6)]
    write_gguf(path, md, tensors)
    return path
