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

import glob
import json
import os

import torch

from ..models.llama import LayerWeights, LlamaModel


def resolve_checkpoint_dir(model: str) -> str:
    if os.path.isdir(model):
        return model
    from ..config import _hf_cache_dir

    d = _hf_cache_dir(model)
    if d and glob.glob(os.path.join(d, "*.safetensors")):
        return d
    try:  # first start of a pod: populate the PVC-backed HF cache
        from huggingface_hub import snapshot_download

        return snapshot_download(model, allow_patterns=["*.json", "*.safetensors", "tokenizer*"],
                                 token=os.environ.get("HUGGING_FACE_HUB_TOKEN"))
    except Exception as e:  # pragma: no cover - no network in CI
        raise FileNotFoundError(f"checkpoint {model!r} not found locally and download failed: {e}")


class _Ckpt:
    def __init__(self, path: str):
        from safetensors import safe_open

        files = sorted(glob.glob(os.path.join(path, "*.safetensors")))
        if not files:
            raise FileNotFoundError(f"no *.safetensors in {path}")
        self.handles = [safe_open(f, framework="pt") for f in files]
        self.where = {}
        for h in self.handles:
            for k in h.keys():
                self.where[k] = h

    def has(self, name):
        return name in self.where

    def full(self, name) -> torch.Tensor:
        return self.where[name].get_tensor(name)

    def rows(self, name, start, stop) -> torch.Tensor:
        return self.where[name].get_slice(name)[start:stop]

    def cols(self, name, start, stop) -> torch.Tensor:
        return self.where[name].get_slice(name)[:, start:stop]


def load_hf_weights(model: LlamaModel, model_path: str):
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

    def to(t):
        return t.to(device=dev, dtype=dt).contiguous()

    def vocab_shard(name):
        t = ck.rows(name, r * vpad, min((r + 1) * vpad, cfg.vocab_size))
        if t.shape[0] < vpad:
            t = torch.cat([t, torch.zeros(vpad - t.shape[0], H, dtype=t.dtype)])
        return to(t)

    model.embed = vocab_shard("model.embed_tokens.weight")
    model.norm = to(ck.full("model.norm.weight"))
    if cfg.tie_word_embeddings or not ck.has("lm_head.weight"):
        model.lm_head = model.embed
    else:
        model.lm_head = vocab_shard("lm_head.weight")
    model.layers = []
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        q = ck.rows(p + "self_attn.q_proj.weight", r * nq * D, (r + 1) * nq * D)
        k = ck.rows(p + "self_attn.k_proj.weight", kv0 * D, (kv0 + nkv) * D)
        v = ck.rows(p + "self_attn.v_proj.weight", kv0 * D, (kv0 + nkv) * D)
        lw = LayerWeights(
            ln1=to(ck.full(p + "input_layernorm.weight")),
            wqkv=to(torch.cat([q, k, v], 0)),
            wo=to(ck.cols(p + "self_attn.o_proj.weight", r * nq * D, (r + 1) * nq * D)),
            ln2=to(ck.full(p + "post_attention_layernorm.weight")),
        )
        if cfg.num_experts:
            E = cfg.num_experts
            m = p + "block_sparse_moe."
            lw.router = to(ck.full(m + "gate.weight"))
            w13, w2 = [], []
            for e in range(E):
                ep = f"{m}experts.{e}."
                g = ck.rows(ep + "w1.weight", r * inter, (r + 1) * inter)
                u = ck.rows(ep + "w3.weight", r * inter, (r + 1) * inter)
                w13.append(torch.cat([g, u], 0))
                w2.append(ck.cols(ep + "w2.weight", r * inter, (r + 1) * inter))
            lw.w13 = to(torch.stack(w13))
            lw.w2 = to(torch.stack(w2))
        else:
            g = ck.rows(p + "mlp.gate_proj.weight", r * inter, (r + 1) * inter)
            u = ck.rows(p + "mlp.up_proj.weight", r * inter, (r + 1) * inter)
            lw.wgu = to(torch.cat([g, u], 0))
            lw.wd = to(ck.cols(p + "mlp.down_proj.weight", r * inter, (r + 1) * inter))
        model.layers.append(lw)


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
