"""Model and engine configuration.

``ModelConfig`` mirrors the fields of a HuggingFace ``config.json`` (Llama /
Mixtral families) and of GGUF ``llama.*`` metadata. ``EngineConfig`` carries the
flags the reference charts pass to the engine
(``vllm-models/helm-chart/templates/model-deployments.yaml:26-39``:
``--model --served-model-name --gpu-memory-utilization --tensor-parallel-size``)
plus the ``llama-server`` flags of the GGUF tier
(``ramalama-models/helm-chart/templates/model-deployments.yaml:26-35``).
Both are frozen after construction: no global mutable flags.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field


@dataclass(frozen=True)
class ModelConfig:
    name: str = "llama"
    architecture: str = "llama"          # llama | mixtral
    hidden_size: int = 4096
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    intermediate_size: int = 14336
    vocab_size: int = 128256
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: dict | None = None
    rope_mode: int = 0                    # 0 NeoX rotate-half (HF), 1 interleaved (GGUF)
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False
    num_experts: int = 0
    num_experts_per_tok: int = 0
    bos_token_id: int | None = 128000
    eos_token_id: tuple = (128001, 128009)

    @property
    def q_size(self):
        return self.num_heads * self.head_dim

    @property
    def kv_size(self):
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        H, I, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        mlp = 3 * H * I * max(1, self.num_experts) + (H * self.num_experts if self.num_experts else 0)
        emb = V * H * (1 if self.tie_word_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H

    @staticmethod
    def from_hf_dict(d: dict, name: str = "model") -> "ModelConfig":
        arch = (d.get("architectures") or ["LlamaForCausalLM"])[0]
        family = "mixtral" if "Mixtral" in arch or d.get("num_local_experts") else "llama"
        nh = d["num_attention_heads"]
        H = d["hidden_size"]
        eos = d.get("eos_token_id", 2)
        eos = tuple(eos) if isinstance(eos, (list, tuple)) else (eos,)
        return ModelConfig(
            name=name,
            architecture=family,
            hidden_size=H,
            num_layers=d["num_hidden_layers"],
            num_heads=nh,
            num_kv_heads=d.get("num_key_value_heads", nh),
            head_dim=d.get("head_dim") or H // nh,
            intermediate_size=d["intermediate_size"],
            vocab_size=d["vocab_size"],
            rms_norm_eps=d.get("rms_norm_eps", 1e-5),
            rope_theta=d.get("rope_theta", 10000.0),
            rope_scaling=d.get("rope_scaling"),
            max_position_embeddings=d.get("max_position_embeddings", 4096),
            tie_word_embeddings=d.get("tie_word_embeddings", False),
            num_experts=d.get("num_local_experts", 0) or 0,
            num_experts_per_tok=d.get("num_experts_per_tok", 0) or 0,
            bos_token_id=d.get("bos_token_id"),
            eos_token_id=eos,
        )

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


_LLAMA3_SCALING = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                   "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}

# Public architecture hyper-parameters. Random-init weights of these
# shapes are what the benchmarks run (no network => no checkpoints).
PRESETS: dict[str, ModelConfig] = {
    "llama-3-8b": ModelConfig(name="llama-3-8b", hidden_size=4096, num_layers=32, num_heads=32,
                              num_kv_heads=8, intermediate_size=14336, vocab_size=128256,
                              rope_theta=500000.0, max_position_embeddings=8192),
    "llama-3.1-8b": ModelConfig(name="llama-3.1-8b", hidden_size=4096, num_layers=32, num_heads=32,
                                num_kv_heads=8, intermediate_size=14336, vocab_size=128256,
                                rope_theta=500000.0, rope_scaling=_LLAMA3_SCALING,
                                max_position_embeddings=131072),
    "llama-3-70b": ModelConfig(name="llama-3-70b", hidden_size=8192, num_layers=80, num_heads=64,
                               num_kv_heads=8, intermediate_size=28672, vocab_size=128256,
                               rope_theta=500000.0, max_position_embeddings=8192),
    "mixtral-8x7b": ModelConfig(name="mixtral-8x7b", architecture="mixtral", hidden_size=4096,
                                num_layers=32, num_heads=32, num_kv_heads=8,
                                intermediate_size=14336, vocab_size=32000, rope_theta=1e6,
                                max_position_embeddings=32768, num_experts=8,
                                num_experts_per_tok=2, bos_token_id=1, eos_token_id=(2,)),
    "tinyllama-1.1b": ModelConfig(name="tinyllama-1.1b", hidden_size=2048, num_layers=22,
                                  num_heads=32, num_kv_heads=4, head_dim=64,
                                  intermediate_size=5632, vocab_size=32000, rope_theta=10000.0,
                                  max_position_embeddings=2048, bos_token_id=1, eos_token_id=(2,)),
    # tiny shapes for CPU plumbing tests
    "tiny-llama": ModelConfig(name="tiny-llama", hidden_size=128, num_layers=2, num_heads=4,
                              num_kv_heads=2, head_dim=32, intermediate_size=256, vocab_size=512,
                              rope_theta=10000.0, max_position_embeddings=2048,
                              bos_token_id=1, eos_token_id=(2,)),
    "tiny-mixtral": ModelConfig(name="tiny-mixtral", architecture="mixtral", hidden_size=128,
                                num_layers=2, num_heads=4, num_kv_heads=2, head_dim=32,
                                intermediate_size=192, vocab_size=512, rope_theta=1e6,
                                max_position_embeddings=2048, num_experts=4,
                                num_experts_per_tok=2, bos_token_id=1, eos_token_id=(2,)),
    # GPU-test sized (head_dim 128 / 64 so the HIP kernels are exercised)
    "small-llama": ModelConfig(name="small-llama", hidden_size=512, num_layers=2, num_heads=8,
                               num_kv_heads=2, head_dim=64, intermediate_size=1024,
                               vocab_size=1024, rope_theta=10000.0, max_position_embeddings=4096,
                               bos_token_id=1, eos_token_id=(2,)),
    "small-mixtral": ModelConfig(name="small-mixtral", architecture="mixtral", hidden_size=512,
                                 num_layers=2, num_heads=8, num_kv_heads=2, head_dim=64,
                                 intermediate_size=768, vocab_size=1024, rope_theta=1e6,
                                 max_position_embeddings=4096, num_experts=8,
                                 num_experts_per_tok=2, bos_token_id=1, eos_token_id=(2,)),
}


def resolve_model_config(model: str, name: str | None = None) -> ModelConfig:
    """Preset name, HF model directory (config.json), HF cache id, or a .gguf file."""
    key = model.lower().split("/")[-1]
    for k, cfg in PRESETS.items():
        if key == k or key.replace("meta-", "").replace("-instruct", "") == k:
            return cfg
    if os.path.isdir(model) and os.path.exists(os.path.join(model, "config.json")):
        with open(os.path.join(model, "config.json")) as f:
            return ModelConfig.from_hf_dict(json.load(f), name=name or os.path.basename(model))
    if model.endswith(".gguf") and os.path.exists(model):
        from .weights.gguf import GGUFFile

        return GGUFFile(model).model_config(name=name)
    hub = _hf_cache_dir(model)
    if hub:
        with open(os.path.join(hub, "config.json")) as f:
            return ModelConfig.from_hf_dict(json.load(f), name=name or model)
    raise ValueError(f"unknown model {model!r}: not a preset ({', '.join(PRESETS)}), "
                     "a directory with config.json, a cached HF id or a .gguf file")


def _hf_cache_dir(repo_id: str) -> str | None:
    """Locate a snapshot of an HF Hub repo in the local cache (offline)."""
    if "/" not in repo_id:
        return None
    home = os.environ.get("HF_HOME", os.path.expanduser("~/.cache/huggingface"))
    base = os.path.join(home, "hub", "models--" + repo_id.replace("/", "--"), "snapshots")
    if not os.path.isdir(base):
        return None
    for snap in sorted(os.listdir(base)):
        p = os.path.join(base, snap)
        if os.path.exists(os.path.join(p, "config.json")):
            return p
    return None


@dataclass(frozen=True)
class EngineConfig:
    model: str = "llama-3-8b"
    served_model_name: str | None = None
    tokenizer: str | None = None
    load_format: str = "auto"            # auto | dummy | safetensors | gguf
    dtype: str = "bfloat16"
    device: str = "cuda"
    tensor_parallel_size: int = 1
    gpu_memory_utilization: float = 0.90
    max_model_len: int | None = None
    block_size: int = 16
    max_num_seqs: int = 256
    max_num_batched_tokens: int = 8192
    num_kv_blocks: int | None = None     # override the memory-derived KV pool size
    enable_prefix_caching: bool = True
    enforce_eager: bool = False
    cuda_graph_max_bs: int = 256
    seed: int = 0
    trust_remote_code: bool = False
    decode_partition: int = 512
    host: str = "0.0.0.0"
    port: int = 8080
    extra: dict = field(default_factory=dict)

    def replace(self, **kw) -> "EngineConfig":
        return dataclasses.replace(self, **kw)

    @property
    def model_name(self) -> str:
        return self.served_model_name or self.model
