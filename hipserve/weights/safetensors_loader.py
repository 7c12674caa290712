"""HuggingFace safetensors checkpoint loader with tensor-parallel slicing.

Each TP rank reads only its own shard of every tensor (``safe_open(...).get_slice``
memory-maps the file; no full-tensor materialisation), merges q/k/v and gate/up
into the fused layouts the kernels use, and moves the result to its GPU in bf16.
Resolves ``--model`` as a local directory or an HF Hub id in the local cache
(the chart mounts the per-model PVC at ``/root/.cache/huggingface`` —
vllm-models/helm-chart/templates/model-deployments.yaml:45-47), downloading with
``huggingface_hub.snapshot_download`` only when the cache is empty and the
network is reachable.
"""
from __future__ import annotations

import json
import os

import torch

from ..models.llama import LayerWeights, LlamaModel


def resolve_checkpoint_dir(model: str) -> str:
    if os.path.isdir(model):
        return model
    from ..config import _hf_cache_dir

    from .hub import download, snapshot_problem

    d = _hf_cache_dir(model)
    if snapshot_problem(d, True) is None:
        return d
    try:  # normally materialised by prepare_model already; resumes a partial snapshot
        return download(model, True)
    except Exception as e:  # pragma: no cover - no network in CI
        raise FileNotFoundError(f"checkpoint {model!r} not found locally and download failed: {e}")


class _Ckpt:
    def __init__(self, path: str):
        from safetensors import safe_open

        from .hub import weight_files

        files = weight_files(path)  # the index's shard list when there is one
        if not files:
            raise FileNotFoundError(f"no *.safetensors in {path}")
        missing = [os.path.basename(f) for f in files if not os.path.exists(f)]
        if missing:
            raise FileNotFoundError(f"{path}: shards listed in the index are missing: {', '.join(missing)}")
        self.handles = [safe_open(f, framework="pt") for f in files]
        self.where = {}
        for h in self.handles:
            for k in h.keys():
                self.where[k] = h
        # integer weight-only checkpoints (weights/int_quant.py): "<x>.weight" is a
        # virtual tensor dequantised from "<x>.weight_packed" / "<x>.qweight"
        self.bits = _quant_bits(path)
        self.virtual = {}
        for k in list(self.where):
            for suf, kind in ((".weight_packed", "ct"), (".qweight", "awq")):
                if k.endswith(suf) and k[: -len(suf)] + ".weight" not in self.where:
                    self.virtual[k[: -len(suf)] + ".weight"] = (kind, k[: -len(suf)])

    def has(self, name):
        return name in self.where or name in self.virtual

    def find(self, suffix) -> str | None:
        for k in list(self.where) + list(self.virtual):
            if k.endswith(suffix):
                return k
        return None

    def _get(self, name):
        return self.where[name].get_tensor(name) if name in self.where else None

    def full(self, name) -> torch.Tensor:
        if name in self.virtual:
            return self._dequant_int(name)
        t = self.where[name].get_tensor(name)
        return self._dequant(name, t) if t.dtype in _FP8 else t

    def rows(self, name, start, stop) -> torch.Tensor:
        if self._is_fp8(name):
            return self.full(name)[start:stop]
        return self.where[name].get_slice(name)[start:stop]

    def cols(self, name, start, stop) -> torch.Tensor:
        if self._is_fp8(name):
            return self.full(name)[:, start:stop]
        return self.where[name].get_slice(name)[:, start:stop]

    # ---- native FP8: e4m3 bits + scale, sliced per TP rank, never dequantised
    def fp8_scale_name(self, name) -> str | None:
        base = name[: -len("weight")] if name.endswith("weight") else name + "_"
        for sname in (base + "weight_scale", base + "weight_scale_inv"):
            if sname in self.where:
                return sname
        return None

    def is_fp8_e4m3(self, name) -> bool:
        return (name in self.where and self.where[name].get_slice(name).get_dtype() == "F8_E4M3"
                and self.fp8_scale_name(name) is not None)

    def fp8_part(self, name, axis: int, start: int, stop: int):
        """(e4m3 weight slice, matching scale) — rows (axis 0, output channels) or
        columns (axis 1, input features) [start, stop). None when a 128-block scale
        would need a split block."""
        sname = self.fp8_scale_name(name)
        sc = self.where[sname].get_tensor(sname).float()
        sl = self.where[name].get_slice(name)
        q = sl[start:stop] if axis == 0 else sl[:, start:stop]
        per_row = sc.numel() == 1 or (sc.dim() >= 1 and sc.shape[0] == sl.get_shape()[0] and sc.numel() == sc.shape[0])
        if per_row:
            return q, (sc.reshape(-1)[start:stop] if axis == 0 and sc.numel() > 1 else sc.reshape(-1))
        if start % 128:
            return None
        b0, b1 = start // 128, -(-stop // 128)
        return q, (sc[b0:b1] if axis == 0 else sc[:, b0:b1])

    # ---- native 8-bit integer weight-only (compressed-tensors pack-quantized, 8 bits)
    def is_int8_ct(self, name) -> bool:
        return self.bits == 8 and self.virtual.get(name, (None,))[0] == "ct"

    def int8_part(self, name, axis: int, start: int, stop: int):
        """(unsigned bytes q + 128 [rows, cols], scale, zero point or None) of rows /
        columns [start, stop); None when a column slice would split a group."""
        from . import int_quant

        base = self.virtual[name][1]
        packed = self._get(base + ".weight_packed")
        scale = self._get(base + ".weight_scale").float()
        zp = self._get(base + ".weight_zero_point")
        shp = self._get(base + ".weight_shape")
        N = packed.shape[0]
        K = int(shp.reshape(-1)[1]) if shp is not None else packed.shape[1] * 4
        u = int_quant._unpack_rows(packed, 8, K).to(torch.uint8)
        if scale.dim() == 1:
            scale = scale.reshape(-1, 1)
        if zp is not None:
            if zp.dtype == torch.int32 and zp.shape[0] != N:  # packed along N
                zp = (int_quant._unpack_rows(zp.t().contiguous(), 8, N) - 128).t()
            zp = zp.float().reshape(N, -1)
        if axis == 0:
            return u[start:stop], scale[start:stop], (zp[start:stop] if zp is not None else None)
        G = K // scale.shape[1]
        if scale.shape[1] > 1 and (start % G or stop % G):
            return None
        cs = slice(start // G, stop // G) if scale.shape[1] > 1 else slice(0, 1)
        return u[:, start:stop], scale[:, cs], (zp[:, cs] if zp is not None else None)

    def _is_fp8(self, name) -> bool:
        """True for every tensor that must be dequantised whole before slicing."""
        if name in self.virtual:
            return True
        return self.where[name].get_slice(name).get_dtype() in ("F8_E4M3", "F8_E5M2")

    def _dequant_int(self, name) -> torch.Tensor:
        from . import int_quant

        kind, base = self.virtual[name]
        if kind == "awq":
            return int_quant.dequant_awq(self._get(base + ".qweight"), self._get(base + ".qzeros"),
                                         self._get(base + ".scales"))
        return int_quant.dequant_pack_quantized(
            self._get(base + ".weight_packed"), self._get(base + ".weight_scale"),
            self._get(base + ".weight_zero_point"), self._get(base + ".weight_shape"), self.bits)

    def _dequant(self, name, t) -> torch.Tensor:
        """FP8 checkpoints (compressed-tensors "FP8-Dynamic" / block-FP8): weights
        are dequantised to the compute dtype at load with their ``weight_scale``
        (per tensor or per output channel) or ``weight_scale_inv`` (128x128 blocks)."""
        base = name[: -len("weight")] if name.endswith("weight") else name + "_"
        for sname in (base + "weight_scale", base + "weight_scale_inv"):
            if sname in self.where:
                s = self.where[sname].get_tensor(sname).float()
                w = t.float()
                if s.numel() == 1 or (s.dim() >= 1 and s.shape[0] == w.shape[0] and s.numel() == w.shape[0]):
                    return w * s.reshape(-1, *([1] * (w.dim() - 1))) if s.numel() > 1 else w * s.reshape(())
                bn, bk = -(-w.shape[0] // s.shape[0]), -(-w.shape[1] // s.shape[1])
                s = s.repeat_interleave(bn, 0)[: w.shape[0]].repeat_interleave(bk, 1)[:, : w.shape[1]]
                return w * s
        raise ValueError(f"FP8 tensor {name} without weight_scale / weight_scale_inv")


def _quant_bits(path: str) -> int | None:
    """Weight bit width from config.json's quantization_config (compressed-tensors
    ``config_groups.*.weights.num_bits`` or AWQ ``bits``); None if absent."""
    try:
        with open(os.path.join(path, "config.json")) as f:
            q = json.load(f).get("quantization_config") or {}
    except (OSError, ValueError):
        return None
    for grp in (q.get("config_groups") or {}).values():
        w = grp.get("weights") or {}
        if w.get("num_bits"):
            return int(w["num_bits"])
    return int(q["bits"]) if q.get("bits") else None


_FP8 = tuple(getattr(torch, n) for n in ("float8_e4m3fn", "float8_e5m2") if hasattr(torch, n))


def load_hf_weights(model: LlamaModel, model_path: str):
    """Load a HF-format checkpoint of any served family into ``model`` (this rank's
    TP shard): Llama / Mistral, Mixtral, Qwen2 (q/k/v bias), Qwen3 (q/k norms),
    Qwen3-MoE (incl. the fused, transposed expert tensors of Qwen3-VL-MoE), Gemma-3
    text (sandwich norms stored as fp32 ``1 + w``), Phi-3 (fused qkv / gate_up).
    Multimodal wrappers are read through their language-model prefix."""
    ck = _Ckpt(resolve_checkpoint_dir(model_path))
    cfg, tp = model.cfg, model.tp
    r, W = tp.rank, tp.world_size
    D, H = cfg.head_dim, cfg.hidden_size
    dev, dt = model.device, model.dtype
    nq, nkv, inter, vpad = model.nq, model.nkv, model.inter, model.vpad
    if cfg.num_kv_heads >= W:
        kv0 = r * nkv
    else:  # replicated kv heads: rank r uses kv head r // (W / nkv_total)
        kv0 = r // (W // cfg.num_kv_heads)
    emb_name = ck.find("embed_tokens.weight")
    if emb_name is None:
        raise KeyError("no embed_tokens.weight in the checkpoint")
    pre = emb_name[: -len("embed_tokens.weight")]  # "model." | "model.language_model." | ...

    def to(t):
        return t.to(device=dev, dtype=dt).contiguous()

    # native FP8 projections (the FP8-Dynamic / block-FP8 checkpoints, e4m3 + scales)
    # and 8-bit integer weight-only projections (compressed-tensors pack-quantized,
    # the reference's AWQ-8bit export) stay quantised in HBM and are multiplied by
    # the v2 dequant-MFMA kernel (ops/quant.py): half the bytes of bf16 weights
    native_fp8 = dev.type == "cuda" and getattr(model, "native_fp8", True)
    n_fp8 = [0]

    def proj(specs):
        """specs: [(name, axis, start, stop)] stacked along the output rows."""
        if native_fp8 and all(ck.is_fp8_e4m3(n) for n, *_ in specs):
            from ..ops import quant as Q

            parts = [ck.fp8_part(n, ax, a, b) for n, ax, a, b in specs]
            if all(pp is not None for pp in parts) and all(
                    pp[0].shape[0] % 16 == 0 and pp[0].shape[1] % 256 == 0 for pp in parts):
                n_fp8[0] += 1
                return Q.QuantWeight([Q.QuantPart.from_fp8(qq, sc, dev) for qq, sc in parts])
        if native_fp8 and all(ck.is_int8_ct(n) for n, *_ in specs):
            from ..ops import quant as Q

            parts = [ck.int8_part(n, ax, a, b) for n, ax, a, b in specs]
            if all(pp is not None for pp in parts) and all(
                    pp[0].shape[0] % 16 == 0 and pp[0].shape[1] % 256 == 0
                    and (pp[0].shape[1] // pp[1].shape[1]) % 32 == 0 for pp in parts):
                n_fp8[0] += 1
                return Q.QuantWeight([Q.QuantPart.from_int8(u, sc, zp, dev) for u, sc, zp in parts])
        ts = [ck.rows(n, a, b) if ax == 0 else ck.cols(n, a, b) for n, ax, a, b in specs]
        return to(torch.cat(ts, 0) if len(ts) > 1 else ts[0])

    def normw(name):
        """RMSNorm weight: Gemma's x * (1 + w) kept exactly as fp32 (1 + w)."""
        t = ck.full(name)
        if cfg.norm_offset:
            return (1.0 + t.float()).to(device=dev).contiguous()
        return to(t)

    def headnorm(name):  # q/k norms: fp32 weights for the per-head RMSNorm op
        t = ck.full(name).float()
        return ((1.0 + t) if cfg.norm_offset else t).to(device=dev).contiguous()

    def vocab_shard(name):
        t = ck.rows(name, r * vpad, min((r + 1) * vpad, cfg.vocab_size))
        if t.shape[0] < vpad:
            t = torch.cat([t, torch.zeros(vpad - t.shape[0], H, dtype=t.dtype)])
        return to(t)

    model.embed = vocab_shard(emb_name)
    model.norm = normw(pre + "norm.weight")
    head = "lm_head.weight" if ck.has("lm_head.weight") else ck.find("lm_head.weight")
    if cfg.tie_word_embeddings or head is None:
        model.lm_head = model.embed
    else:
        model.lm_head = vocab_shard(head)
    qs, ks = (slice(r * nq * D, (r + 1) * nq * D), slice(kv0 * D, (kv0 + nkv) * D))
    model.layers = []
    for i in range(cfg.num_layers):
        p = f"{pre}layers.{i}."
        a = p + "self_attn."
        if ck.has(a + "qkv_proj.weight"):  # Phi-3: fused [q; k; v]
            f = ck.full(a + "qkv_proj.weight")
            q, k, v = torch.split(f, [cfg.num_heads * D, cfg.num_kv_heads * D, cfg.num_kv_heads * D], 0)
            q, k, v = q[qs], k[ks], v[ks]
            wqkv = to(torch.cat([q, k, v], 0))
        else:
            wqkv = proj([(a + "q_proj.weight", 0, qs.start, qs.stop), (a + "k_proj.weight", 0, ks.start, ks.stop),
                         (a + "v_proj.weight", 0, ks.start, ks.stop)])
        lw = LayerWeights(
            ln1=normw(p + "input_layernorm.weight"),
            wqkv=wqkv,
            wo=proj([(a + "o_proj.weight", 1, qs.start, qs.stop)]),
            ln2=normw(p + ("pre_feedforward_layernorm.weight" if cfg.sandwich_norm
                           else "post_attention_layernorm.weight")),
        )
        if cfg.qkv_bias:
            lw.bqkv = to(torch.cat([ck.full(a + "q_proj.bias")[qs], ck.full(a + "k_proj.bias")[ks],
                                    ck.full(a + "v_proj.bias")[ks]], 0))
        if cfg.qk_norm:
            lw.q_norm = headnorm(a + "q_norm.weight")
            lw.k_norm = headnorm(a + "k_norm.weight")
        if cfg.sandwich_norm:
            lw.post_attn_norm = normw(p + "post_attention_layernorm.weight")
            lw.post_ff_norm = normw(p + "post_feedforward_layernorm.weight")
        if cfg.num_experts:
            lw.router, lw.w13, lw.w2 = _load_experts(ck, p, cfg, r, inter, to, dev if native_fp8 else None)
        elif ck.has(p + "mlp.gate_up_proj.weight"):  # Phi-3: fused [gate; up]
            f = ck.full(p + "mlp.gate_up_proj.weight")
            I = cfg.intermediate_size
            lw.wgu = to(torch.cat([f[r * inter:(r + 1) * inter], f[I + r * inter:I + (r + 1) * inter]], 0))
            lw.wd = to(ck.cols(p + "mlp.down_proj.weight", r * inter, (r + 1) * inter))
        else:
            lw.wgu = proj([(p + "mlp.gate_proj.weight", 0, r * inter, (r + 1) * inter),
                           (p + "mlp.up_proj.weight", 0, r * inter, (r + 1) * inter)])
            lw.wd = proj([(p + "mlp.down_proj.weight", 1, r * inter, (r + 1) * inter)])
        model.layers.append(lw)
    if n_fp8[0]:
        from ..ops import quant as Q

        model.quant_linear = Q.quant_linear
    if model.visual is not None:  # Qwen3-VL vision tower (bf16 in every checkpoint, replicated)
        vname = ck.find("patch_embed.proj.weight")
        if vname is None:
            raise KeyError("vision config present but no visual.patch_embed.proj.weight in the checkpoint")
        model.visual.load(ck.full, vname[: -len("patch_embed.proj.weight")])


def _load_experts(ck, p, cfg, r, inter, to, native_dev=None):
    """(router [E, H], w13 [E, 2*I/TP, H] as [gate; up], w2 [E, H, I/TP]) from
    Mixtral (block_sparse_moe.experts.e.w1/w3/w2), Qwen3-MoE
    (mlp.experts.e.gate_proj/up_proj/down_proj) or fused expert tensors
    (mlp.experts.gate_up_proj [E, 2I, H] / Qwen3-VL-MoE's transposed [E, H, 2I]).
    With ``native_dev`` (a GPU), per-expert INT8 (compressed-tensors 8-bit, the
    reference's AWQ-8bit export) or per-channel FP8 experts stay quantised
    (``QuantMoE`` stacks for the quantised expert GEMM) instead of becoming bf16."""
    E, H, I = cfg.num_experts, cfg.hidden_size, cfg.expert_size
    sl = slice(r * inter, (r + 1) * inter)
    if ck.has(p + "block_sparse_moe.gate.weight"):
        m = p + "block_sparse_moe."
        names = ("w1", "w3", "w2")
    else:
        m = p + "mlp."
        names = ("gate_proj", "up_proj", "down_proj")
    router = to(ck.full(m + "gate.weight"))
    if native_dev is not None and not ck.has(m + "experts.gate_up_proj"):
        q = _native_experts(ck, m, names, E, sl, native_dev)
        if q is not None:
            return router, q[0], q[1]
    if ck.has(m + "experts.gate_up_proj"):
        gu = ck.full(m + "experts.gate_up_proj")
        dn = ck.full(m + "experts.down_proj")
        if tuple(gu.shape) == (E, H, 2 * I) and (H != 2 * I or cfg.family == "qwen3_moe"):
            gu = gu.transpose(1, 2)
        if tuple(dn.shape) == (E, I, H) and (H != I or cfg.family == "qwen3_moe"):
            dn = dn.transpose(1, 2)
        w13 = torch.cat([gu[:, sl], gu[:, I + sl.start:I + sl.stop]], 1)
        w2 = dn[:, :, sl]
        return router, to(w13), to(w2)
    w13, w2 = [], []
    for e in range(E):
        ep = f"{m}experts.{e}."
        g = ck.rows(ep + names[0] + ".weight", sl.start, sl.stop)
        u = ck.rows(ep + names[1] + ".weight", sl.start, sl.stop)
        w13.append(torch.cat([g, u], 0))
        w2.append(ck.cols(ep + names[2] + ".weight", sl.start, sl.stop))
    return router, to(torch.stack(w13)), to(torch.stack(w2))


def _native_experts(ck, m, names, E, sl, dev):
    """(QuantMoE w13, QuantMoE w2) of per-expert INT8 / per-channel FP8 tensors, or None
    when the experts are another format or a slice would split a scale group."""
    from ..ops import quant as Q

    first = f"{m}experts.0.{names[0]}.weight"
    int8 = ck.is_int8_ct(first)
    if not int8 and not ck.is_fp8_e4m3(first):
        return None

    def part(name, axis):
        pp = ck.int8_part(name, axis, sl.start, sl.stop) if int8 else ck.fp8_part(name, axis, sl.start, sl.stop)
        if pp is None or (not int8 and pp[1].numel() not in (1, pp[0].shape[0])):
            raise ValueError("unsupported expert slice")  # a split group / 128-block scales
        return pp

    def build(pps, channel=True):  # row-stacked pieces of one expert -> QuantPart
        if int8:
            zps = [z for _, _, z in pps]
            zp = None if all(z is None for z in zps) else torch.cat(
                [z if z is not None else torch.zeros_like(sc) for (_, sc, _), z in zip(pps, zps)])
            return Q.QuantPart.from_int8(torch.cat([u for u, _, _ in pps]), torch.cat([sc for _, sc, _ in pps]),
                                         zp, dev, channel)
        qs = torch.cat([q for q, _ in pps])
        sc = torch.cat([s.reshape(-1).expand(q.shape[0]) if s.numel() == 1 else s.reshape(-1) for q, s in pps])
        return Q.QuantPart.from_fp8(qs, sc, dev)

    try:
        p13, p2 = [], []
        for e in range(E):
            ep = f"{m}experts.{e}."
            p13.append(build([part(ep + names[0] + ".weight", 0), part(ep + names[1] + ".weight", 0)]))
            p2.append(build([part(ep + names[2] + ".weight", 1)]))
        if int8 and len({p.kqt for p in p13 + p2}) > 1:  # zero points on some experts only: one format
            p13 = [build([part(f"{m}experts.{e}." + names[0] + ".weight", 0),
                          part(f"{m}experts.{e}." + names[1] + ".weight", 0)], False) for e in range(E)]
            p2 = [build([part(f"{m}experts.{e}." + names[2] + ".weight", 1)], False) for e in range(E)]
    except ValueError:
        return None
    if not (Q.QuantMoE.supported(p13[0].kqt, p13[0].N, p13[0].K) and Q.QuantMoE.supported(p2[0].kqt, p2[0].N, p2[0].K)):
        return None
    return Q.QuantMoE(p13, kmajor=True), Q.QuantMoE(p2)


def save_hf_checkpoint(path: str, cfg, tensors: dict[str, torch.Tensor]):
    """Write a minimal HF-format checkpoint (config.json + model.safetensors);
    used by tests and by `hipserve.weights.export`."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    arch = "MixtralForCausalLM" if cfg.num_experts else "LlamaForCausalLM"
    conf = {"architectures": [arch], "hidden_size": cfg.hidden_size,
            "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
            "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
            "intermediate_size": cfg.intermediate_size, "vocab_size": cfg.vocab_size,
            "rms_norm_eps": cfg.rms_norm_eps, "rope_theta": cfg.rope_theta,
            "max_position_embeddings": cfg.max_position_embeddings,
            "tie_word_embeddings": cfg.tie_word_embeddings, "bos_token_id": cfg.bos_token_id,
            "eos_token_id": list(cfg.eos_token_id), "torch_dtype": "bfloat16"}
    if cfg.rope_scaling:
        conf["rope_scaling"] = cfg.rope_scaling
    if cfg.num_experts:
        conf["num_local_experts"] = cfg.num_experts
        conf["num_experts_per_tok"] = cfg.num_experts_per_tok
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(conf, f, indent=1)
    save_file({k: v.contiguous() for k, v in tensors.items()}, os.path.join(path, "model.safetensors"))


def random_hf_tensors(cfg, seed: int = 0, std: float = 0.05) -> dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    H, D, I, V = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size, cfg.vocab_size

    def rnd(*s):
        return torch.randn(*s, generator=g) * std

    t = {"model.embed_tokens.weight": rnd(V, H), "model.norm.weight": 1 + rnd(H),
         "lm_head.weight": rnd(V, H)}
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        t[p + "input_layernorm.weight"] = 1 + rnd(H)
        t[p + "post_attention_layernorm.weight"] = 1 + rnd(H)
        t[p + "self_attn.q_proj.weight"] = rnd(cfg.num_heads * D, H)
        t[p + "self_attn.k_proj.weight"] = rnd(cfg.num_kv_heads * D, H)
        t[p + "self_attn.v_proj.weight"] = rnd(cfg.num_kv_heads * D, H)
        t[p + "self_attn.o_proj.weight"] = rnd(H, cfg.num_heads * D)
        if cfg.num_experts:
            m = p + "block_sparse_moe."
            t[m + "gate.weight"] = rnd(cfg.num_experts, H)
            for e in range(cfg.num_experts):
                t[f"{m}experts.{e}.w1.weight"] = rnd(I, H)
                t[f"{m}experts.{e}.w3.weight"] = rnd(I, H)
                t[f"{m}experts.{e}.w2.weight"] = rnd(H, I)
        else:
            t[p + "mlp.gate_proj.weight"] = rnd(I, H)
            t[p + "mlp.up_proj.weight"] = rnd(I, H)
            t[p + "mlp.down_proj.weight"] = rnd(H, I)
    return t
