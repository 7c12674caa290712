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
class VisionConfig:
    """Qwen3-VL vision tower (HF ``vision_config``): a ViT over 16x16x2 (HxWxT)
    patches with a learned, bilinearly resampled position table, 2D RoPE, a 2x2
    spatial merger into the language model's hidden size and DeepStack features
    (merged outputs of intermediate blocks added to the first decoder layers)."""
    depth: int = 27
    hidden_size: int = 1152
    intermediate_size: int = 4304
    num_heads: int = 16
    patch_size: int = 16
    temporal_patch_size: int = 2
    in_channels: int = 3
    spatial_merge_size: int = 2
    out_hidden_size: int = 2048
    num_position_embeddings: int = 2304
    deepstack_visual_indexes: tuple = (8, 16, 24)
    hidden_act: str = "gelu_pytorch_tanh"
    # special tokens of the language model
    image_token_id: int = 151655
    video_token_id: int = 151656
    vision_start_token_id: int = 151652
    vision_end_token_id: int = 151653
    # image preprocessing (preprocessor_config.json)
    min_pixels: int = 65536
    max_pixels: int = 16777216
    image_mean: tuple = (0.5, 0.5, 0.5)
    image_std: tuple = (0.5, 0.5, 0.5)

    @property
    def head_dim(self) -> int:
        return self.hidden_size // self.num_heads

    @property
    def patch_dim(self) -> int:
        return self.in_channels * self.temporal_patch_size * self.patch_size ** 2

    @staticmethod
    def from_hf_dict(d: dict) -> "VisionConfig | None":
        v = d.get("vision_config")
        if not isinstance(v, dict) or "depth" not in v:
            return None
        kw = {k: v[k] for k in ("depth", "hidden_size", "intermediate_size", "num_heads", "patch_size",
                                "temporal_patch_size", "in_channels", "spatial_merge_size", "out_hidden_size",
                                "num_position_embeddings", "hidden_act") if k in v}
        kw["deepstack_visual_indexes"] = tuple(v.get("deepstack_visual_indexes") or ())
        for k in ("image_token_id", "video_token_id", "vision_start_token_id", "vision_end_token_id"):
            if d.get(k) is not None:
                kw[k] = int(d[k])
        return VisionConfig(**kw)


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
    # ---- family options (Qwen2/Qwen3/Qwen3-MoE/Gemma-3/Phi-3; defaults = Llama/Mixtral)
    family: str = "llama"                 # llama | mixtral | qwen2 | qwen3 | qwen3_moe | gemma3 | phi3
    qkv_bias: bool = False                # Qwen2: q/k/v projections carry a bias
    qk_norm: bool = False                 # Qwen3 / Gemma-3: per-head RMSNorm of q and k before RoPE
    moe_intermediate_size: int = 0        # expert width when it differs from intermediate_size (Qwen3-MoE)
    norm_topk_prob: bool = True           # renormalise the top-k routing weights (Mixtral: always)
    hidden_act: str = "silu"              # silu | gelu_tanh (Gemma GeGLU)
    sandwich_norm: bool = False           # Gemma-3: RMSNorm on the attention / MLP outputs too
    norm_offset: bool = False             # Gemma RMSNorm: x * (1 + w)
    embed_scale: float = 1.0              # Gemma: embeddings * sqrt(hidden)
    attn_scale: float = 0.0               # softmax scale (0 = 1/sqrt(head_dim)); Gemma: query_pre_attn_scalar^-0.5
    sliding_window: int = 0               # window of the sliding-attention layers (0 = none)
    layer_windows: tuple = ()             # per-layer window (0 = full attention); empty = all full
    rope_local_theta: float = 0.0         # RoPE base of the sliding layers (Gemma-3: 10000; 0 = rope_theta)
    partial_rotary_factor: float = 1.0
    # Qwen3-VL: interleaved multimodal RoPE (rotary pairs split T/H/W by this
    # section table; text tokens have t = h = w so it reduces to plain RoPE)
    mrope_section: tuple = ()
    vision: VisionConfig | None = None

    @property
    def expert_size(self):
        return self.moe_intermediate_size or self.intermediate_size

    def window_of(self, layer: int) -> int:
        return self.layer_windows[layer] if self.layer_windows else 0

    @property
    def q_size(self):
        return self.num_heads * self.head_dim

    @property
    def kv_size(self):
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        H, I, V, L = self.hidden_size, self.intermediate_size, self.vocab_size, self.num_layers
        attn = H * (self.q_size + 2 * self.kv_size) + self.q_size * H
        if self.num_experts:
            mlp = 3 * H * self.expert_size * self.num_experts + H * self.num_experts
        else:
            mlp = 3 * H * I
        emb = V * H * (1 if self.tie_word_embeddings else 2)
        return L * (attn + mlp + 2 * H) + emb + H

    @staticmethod
    def from_hf_dict(d: dict, name: str = "model") -> "ModelConfig":
        """HF ``config.json`` -> ModelConfig for the served families. Multimodal
        wrappers (Gemma3ForConditionalGeneration, Qwen3-VL-MoE) contribute their
        ``text_config`` (the language model; vision towers are not served). Both the
        Hub's ``rope_theta``/``rope_scaling`` keys and the newer ``rope_parameters``
        form (per layer type for Gemma-3) are read."""
        arch = (d.get("architectures") or ["LlamaForCausalLM"])[0]
        mtype = d.get("model_type", "")
        vision = VisionConfig.from_hf_dict(d) if mtype.startswith("qwen3_vl") or "qwen3vl" in arch.lower() else None
        if isinstance(d.get("text_config"), dict):  # multimodal wrapper: the language model
            td = dict(d["text_config"])
            for k in ("eos_token_id", "bos_token_id", "tie_word_embeddings"):
                if k not in td and k in d:
                    td[k] = d[k]
            d = td
            mtype = d.get("model_type", mtype)
        family = _family_of(arch, mtype, d)
        nh = d["num_attention_heads"]
        H = d["hidden_size"]
        D = d.get("head_dim") or H // nh
        eos = d.get("eos_token_id", 2)
        eos = tuple(eos) if isinstance(eos, (list, tuple)) else (eos,)
        L = d["num_hidden_layers"]
        theta, scaling = _rope_params(d, "full_attention" if family == "gemma3" else None)
        kw = dict(
            name=name,
            architecture="mixtral" if family in ("mixtral", "qwen3_moe") else "llama",
            family=family,
            hidden_size=H,
            num_layers=L,
            num_heads=nh,
            num_kv_heads=d.get("num_key_value_heads") or nh,
            head_dim=D,
            intermediate_size=d["intermediate_size"],
            vocab_size=d["vocab_size"],
            rms_norm_eps=d.get("rms_norm_eps", 1e-5),
            rope_theta=theta,
            rope_scaling=scaling,
            max_position_embeddings=d.get("max_position_embeddings", 4096),
            tie_word_embeddings=d.get("tie_word_embeddings", family == "gemma3"),
            bos_token_id=d.get("bos_token_id"),
            eos_token_id=eos,
            partial_rotary_factor=float(d.get("partial_rotary_factor", 1.0) or 1.0),
        )
        if kw["partial_rotary_factor"] != 1.0:
            raise NotImplementedError("partial rotary embeddings are not supported")
        if vision is not None:
            rp = d.get("rope_parameters") or d.get("rope_scaling") or {}
            sec = tuple(int(x) for x in (rp.get("mrope_section") or (24, 20, 20)))
            if rp.get("mrope_interleaved") is False:
                raise NotImplementedError("non-interleaved MRoPE (Qwen2-VL layout) is not supported")
            kw.update(vision=vision, mrope_section=sec)
        if family == "mixtral":
            kw.update(num_experts=d.get("num_local_experts", 0) or 0,
                      num_experts_per_tok=d.get("num_experts_per_tok", 0) or 0)
        elif family == "qwen2":
            kw.update(qkv_bias=True)
        elif family == "qwen3":
            kw.update(qk_norm=True, qkv_bias=bool(d.get("attention_bias", False)))
        elif family == "qwen3_moe":
            if d.get("decoder_sparse_step", 1) != 1 or d.get("mlp_only_layers"):
                raise NotImplementedError("Qwen3-MoE with dense layers (decoder_sparse_step / mlp_only_layers)")
            kw.update(qk_norm=True, qkv_bias=bool(d.get("attention_bias", False)),
                      num_experts=d.get("num_experts") or d["num_local_experts"],
                      num_experts_per_tok=d["num_experts_per_tok"],
                      moe_intermediate_size=d["moe_intermediate_size"],
                      norm_topk_prob=bool(d.get("norm_topk_prob", False)))
        elif family == "gemma3":
            if d.get("final_logit_softcapping") or d.get("attn_logit_softcapping"):
                raise NotImplementedError("logit soft-capping (Gemma-2) is not supported")
            types = d.get("layer_types")
            if not types:
                pat = d.get("sliding_window_pattern", 6)
                types = ["sliding_attention" if (i + 1) % pat else "full_attention" for i in range(L)]
            win = int(d.get("sliding_window") or 0)
            local_theta, _ = _rope_params(d, "sliding_attention")
            kw.update(qk_norm=True, hidden_act="gelu_tanh", sandwich_norm=True, norm_offset=True,
                      embed_scale=float(H) ** 0.5,
                      attn_scale=float(d.get("query_pre_attn_scalar") or D) ** -0.5,
                      sliding_window=win,
                      layer_windows=tuple(win if t == "sliding_attention" else 0 for t in types),
                      rope_local_theta=local_theta)
        return ModelConfig(**kw)

    def replace(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)


def _family_of(arch: str, mtype: str, d: dict) -> str:
    a, t = arch.lower(), (mtype or "").lower()
    if t.startswith("qwen3_moe") or t.startswith("qwen3_vl_moe") or "qwen3moe" in a or "qwen3vlmoe" in a:
        return "qwen3_moe"
    if t.startswith("qwen3") or a.startswith("qwen3"):
        return "qwen3"
    if t.startswith("qwen2") or a.startswith("qwen2"):
        return "qwen2"
    if t.startswith("gemma3") or a.startswith("gemma3"):
        return "gemma3"
    if t == "phi3" or a.startswith("phi3"):
        return "phi3"
    if t == "mixtral" or "mixtral" in a or d.get("num_local_experts"):
        return "mixtral"
    if t in ("llama", "mistral", "") or "llama" in a or "mistral" in a:
        return "llama"
    raise NotImplementedError(f"unsupported architecture {arch!r} (model_type {mtype!r})")


_ROPE_TYPES = (None, "default", "llama3", "linear")


def _rope_params(d: dict, layer_type: str | None) -> tuple[float, dict | None]:
    """(theta, scaling) from the Hub keys (``rope_theta``, ``rope_scaling``,
    Gemma-3 ``rope_local_base_freq``) or the ``rope_parameters`` form (one dict,
    or one per layer type)."""
    rp = d.get("rope_parameters")
    if isinstance(rp, dict) and ("full_attention" in rp or "sliding_attention" in rp):
        rp = rp.get(layer_type or "full_attention")
    local = layer_type == "sliding_attention"
    if isinstance(rp, dict) and "rope_theta" in rp:
        theta = float(rp["rope_theta"])
        scaling = {k: v for k, v in rp.items() if k != "rope_theta"}
    elif local:  # Hub Gemma-3: local layers run plain RoPE on rope_local_base_freq
        theta, scaling = float(d.get("rope_local_base_freq", 10000.0)), None
    else:
        theta, scaling = float(d.get("rope_theta", 10000.0)), d.get("rope_scaling")
    if scaling is not None:
        typ = scaling.get("rope_type", scaling.get("type"))
        if typ not in _ROPE_TYPES:
            raise NotImplementedError(f"RoPE scaling {typ!r} is not supported ({', '.join(map(str, _ROPE_TYPES[1:]))})")
        if typ in (None, "default"):
            scaling = None
    return theta, scaling


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
    # the reference chart's default model families (vllm-models/helm-chart/values.yaml:1-19,
    # ramalama-models/helm-chart/values.yaml:3-19), text models, public hyper-parameters
    "qwen3-0.6b": ModelConfig(name="qwen3-0.6b", family="qwen3", hidden_size=1024, num_layers=28,
                              num_heads=16, num_kv_heads=8, head_dim=128, intermediate_size=3072,
                              vocab_size=151936, rms_norm_eps=1e-6, rope_theta=1e6,
                              max_position_embeddings=40960, tie_word_embeddings=True, qk_norm=True,
                              bos_token_id=None, eos_token_id=(151643, 151645)),
    "qwen3-30b-a3b": ModelConfig(name="qwen3-30b-a3b", architecture="mixtral", family="qwen3_moe",
                                 hidden_size=2048, num_layers=48, num_heads=32, num_kv_heads=4, head_dim=128,
                                 intermediate_size=6144, moe_intermediate_size=768, num_experts=128,
                                 num_experts_per_tok=8, norm_topk_prob=True, vocab_size=151936,
                                 rms_norm_eps=1e-6, rope_theta=1e6, max_position_embeddings=40960,
                                 qk_norm=True, bos_token_id=None, eos_token_id=(151643, 151645)),
    # the reference's default HF model (vllm-models/helm-chart/values.yaml:8-12) with its
    # vision tower: Qwen3-VL-30B-A3B (text = Qwen3-30B-A3B with interleaved MRoPE)
    "qwen3-vl-30b-a3b": ModelConfig(name="qwen3-vl-30b-a3b", architecture="mixtral", family="qwen3_moe",
                                    hidden_size=2048, num_layers=48, num_heads=32, num_kv_heads=4, head_dim=128,
                                    intermediate_size=6144, moe_intermediate_size=768, num_experts=128,
                                    num_experts_per_tok=8, norm_topk_prob=True, vocab_size=151936,
                                    rms_norm_eps=1e-6, rope_theta=5e6, max_position_embeddings=262144,
                                    qk_norm=True, bos_token_id=None, eos_token_id=(151643, 151645),
                                    mrope_section=(24, 20, 20), vision=VisionConfig()),
    "gemma-3-27b": ModelConfig(name="gemma-3-27b", family="gemma3", hidden_size=5376, num_layers=62,
                               num_heads=32, num_kv_heads=16, head_dim=128, intermediate_size=21504,
                               vocab_size=262208, rms_norm_eps=1e-6, rope_theta=1e6,
                               rope_scaling={"rope_type": "linear", "factor": 8.0},
                               max_position_embeddings=131072, tie_word_embeddings=True, qk_norm=True,
                               hidden_act="gelu_tanh", sandwich_norm=True, norm_offset=True,
                               embed_scale=5376 ** 0.5, attn_scale=168 ** -0.5, sliding_window=1024,
                               layer_windows=tuple(1024 if (i + 1) % 6 else 0 for i in range(62)),
                               rope_local_theta=1e4, bos_token_id=2, eos_token_id=(1, 106)),
    "phi-3-mini": ModelConfig(name="phi-3-mini", family="phi3", hidden_size=3072, num_layers=32,
                              num_heads=32, num_kv_heads=32, head_dim=96, intermediate_size=8192,
                              vocab_size=32064, rope_theta=10000.0, max_position_embeddings=4096,
                              bos_token_id=1, eos_token_id=(32000, 32007)),
    # tiny shapes for CPU plumbing tests
    "tiny-llama": ModelConfig(name="tiny-llama", hidden_size=128, num_layers=2, num_heads=4,
                              num_kv_heads=2, head_dim=32, intermediate_size=256, vocab_size=512,
                              rope_theta=10000.0, max_position_embeddings=2048,
                              bos_token_id=1, eos_token_id=(2,)),
    # the 70B head layout in miniature (8 kv heads: one per rank at TP=8) for world-8 CPU runs
    "tiny-llama-tp8": ModelConfig(name="tiny-llama-tp8", hidden_size=256, num_layers=2, num_heads=16,
                                  num_kv_heads=8, head_dim=16, intermediate_size=512, vocab_size=512,
                                  rope_theta=500000.0, max_position_embeddings=2048,
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
    # long-context tests: Llama-3 head geometry (head_dim 128, GQA 4), 64K positions
    "small-llama-long": ModelConfig(name="small-llama-long", hidden_size=1024, num_layers=2, num_heads=8,
                                    num_kv_heads=2, head_dim=128, intermediate_size=2048,
                                    vocab_size=2048, rope_theta=500000.0, max_position_embeddings=65536,
                                    bos_token_id=1, eos_token_id=(2,)),
    "small-mixtral": ModelConfig(name="small-mixtral", architecture="mixtral", hidden_size=512,
                                 num_layers=2, num_heads=8, num_kv_heads=2, head_dim=64,
                                 intermediate_size=768, vocab_size=1024, rope_theta=1e6,
                                 max_position_embeddings=4096, num_experts=8,
                                 num_experts_per_tok=2, bos_token_id=1, eos_token_id=(2,)),
}


def preset_key(model: str) -> str | None:
    """Built-in preset a model name / Hub id maps to (``meta-llama/Meta-Llama-3-8B``
    -> ``llama-3-8b``), or None. Local paths never map to a preset."""
    if os.path.exists(model):
        return None
    key = model.lower().split("/")[-1]
    for k in PRESETS:
        if key == k or key.replace("meta-", "").replace("-instruct", "") == k:
            return k
    return None


def resolve_model_config(model: str, name: str | None = None) -> ModelConfig:
    """Preset name, HF model directory (config.json), HF cache id, or a .gguf file.
    (A Hub id is first materialised into the cache by ``weights.hub.materialize``.)"""
    k = preset_key(model)
    if k is not None and not _hf_cache_dir(model):
        return PRESETS[k]
    if os.path.isdir(model) and os.path.exists(os.path.join(model, "config.json")):
        with open(os.path.join(model, "config.json")) as f:
            return _with_preprocessor(ModelConfig.from_hf_dict(json.load(f), name=name or os.path.basename(model)),
                                      model)
    if model.endswith(".gguf") and os.path.exists(model):
        from .weights.gguf import GGUFFile

        return GGUFFile(model).model_config(name=name)
    hub = _hf_cache_dir(model)
    if hub:
        with open(os.path.join(hub, "config.json")) as f:
            return _with_preprocessor(ModelConfig.from_hf_dict(json.load(f), name=name or model), hub)
    raise ValueError(f"unknown model {model!r}: not a preset ({', '.join(PRESETS)}), "
                     "a directory with config.json, a cached HF id or a .gguf file")


def _with_preprocessor(cfg: ModelConfig, path: str) -> ModelConfig:
    """Image preprocessing limits of a vision model from its preprocessor_config.json
    (``size.shortest_edge`` / ``longest_edge`` or ``min_pixels`` / ``max_pixels``,
    ``image_mean`` / ``image_std``)."""
    p = os.path.join(path, "preprocessor_config.json")
    if cfg.vision is None or not os.path.exists(p):
        return cfg
    with open(p) as f:
        d = json.load(f)
    size = d.get("size") or {}
    kw = {}
    lo = d.get("min_pixels") or size.get("shortest_edge") or size.get("min_pixels")
    hi = d.get("max_pixels") or size.get("longest_edge") or size.get("max_pixels")
    if lo:
        kw["min_pixels"] = int(lo)
    if hi:
        kw["max_pixels"] = int(hi)
    for k in ("image_mean", "image_std"):
        if d.get(k):
            kw[k] = tuple(float(x) for x in d[k])
    if d.get("patch_size") and int(d["patch_size"]) != cfg.vision.patch_size:
        raise ValueError("preprocessor patch_size differs from the vision tower's")
    return cfg.replace(vision=dataclasses.replace(cfg.vision, **kw))


def _hf_cache_dir(repo_id: str) -> str | None:
    """Locate a snapshot of an HF Hub repo in the local cache (offline): the
    revision ``refs/main`` names (what the Hub client resolved last), else the most
    recently written snapshot that has a config.json."""
    if "/" not in repo_id:
        return None
    home = os.environ.get("HF_HOME", os.path.expanduser("~/.cache/huggingface"))
    repo = os.path.join(home, "hub", "models--" + repo_id.replace("/", "--"))
    base = os.path.join(repo, "snapshots")
    if not os.path.isdir(base):
        return None
    try:
        with open(os.path.join(repo, "refs", "main")) as f:
            ref = f.read().strip()
    except OSError:
        ref = ""
    if ref and os.path.exists(os.path.join(base, ref, "config.json")):
        return os.path.join(base, ref)
    snaps = [os.path.join(base, s) for s in os.listdir(base)]
    snaps = [p for p in snaps if os.path.exists(os.path.join(p, "config.json"))]
    return max(snaps, key=lambda p: (os.path.getmtime(p), p)) if snaps else None


GGUF_QUANTS = ("q4_k_m", "q8_0", "q4_0")


def default_batched_tokens(model: str, load_format: str = "auto", quantization: str | None = None) -> int:
    """Prefill token budget per step when none is given: 8192; 16384 for GGUF weights and
    32768 for INT8 weight-only ones. Both keep only their quantised weights and dequantise
    each projection (every expert, for MoE) into a bf16 scratch once per prefill step, a
    cost that more tokens per step spread thinner:
      * Llama-3-8B Q4_K_M: 7,726 -> 8,044 tok/s, p50 TTFT 482 -> 530 ms
        (profiles/r5_bench_q4km_chunk8k.json, r5_bench_q4km_chunk16k.json);
      * Qwen3-30B-A3B INT8 (experts dequantised into the one-launch grouped GEMM's packed
        layout): 4,134 / 646 ms (8K) -> 4,380 / 570 (16K) -> 4,531 / 570 (32K) with a separate
        pack pass, 4,666 / 490 (32K) dequantising straight into the layout; above the
        4,155 / 623 ms of bf16 prefill shadows at 8K with 34 % more KV blocks
        (profiles/r5_bench_q3int8_packed_moe_*.json, r5_bench_q3int8_shadows.json).
    FP8 keeps 8192 (Gemma-3-27B: 2,839 vs 2,854 tok/s at 16K, TTFT 1,110 vs 1,186 ms), and
    so do bf16 MoE models (Mixtral-8x7B: 1,648 / 1,655 / 1,675 tok/s at 8K / 16K / 32K for
    TTFT 558 / 616 / 753 ms, profiles/r5_bench_mixtral*.json). A larger budget also
    lengthens the decode stall of running requests during a prefill step: latency-bound
    deployments pass a smaller --max-num-batched-tokens.
    bf16 models keep 8192: 16384 gave the same 7,730 tok/s at 480 vs 434 ms TTFT and 4096
    7,607 / 432 ms (profiles/r5_bench_8b_chunk16k.json, r5_bench_8b_chunk4k.json)."""
    if quantization is None:
        quantization = checkpoint_quantization(model)
    if quantization == "int8":
        return 32768
    gguf = quantization in GGUF_QUANTS or load_format == "gguf" or str(model).lower().endswith(".gguf")
    return 16384 if gguf else 8192


def checkpoint_quantization(model: str) -> str | None:
    """"int8" / "fp8" from a local HF checkpoint's ``quantization_config`` (compressed-
    tensors weight groups, AWQ / GPTQ bits), else None (presets, Hub ids not yet
    downloaded: the caller's default applies)."""
    path = os.path.join(str(model), "config.json")
    if not os.path.isfile(path):
        return None
    try:
        with open(path) as f:
            q = json.load(f).get("quantization_config") or {}
    except (OSError, ValueError):
        return None
    method = str(q.get("quant_method", "")).lower()
    if method == "fp8":
        return "fp8"
    if method in ("awq", "gptq"):
        return "int8" if int(q.get("bits", 0)) == 8 else None
    for grp in (q.get("config_groups") or {}).values():
        w = (grp or {}).get("weights") or {}
        if int(w.get("num_bits", 0)) == 8:
            return "fp8" if str(w.get("type", "")).lower() == "float" else "int8"
    return None


# --kv-cache-dtype values (vLLM's spellings) -> element kind
KV_CACHE_DTYPES = {"auto": "auto", "bf16": "auto", "bfloat16": "auto", "fp8": "fp8", "fp8_e4m3": "fp8"}


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
    # paged KV cache element: "auto" (= the activation dtype, bf16) or "fp8" / "fp8_e4m3"
    # (OCP e4m3, per-tensor scale 1 as vLLM's --kv-cache-dtype fp8 without calibrated
    # scales: half the KV bytes per token, so 2x the KV blocks and half the decode
    # attention's HBM stream; K / V are rounded to e4m3 when written)
    kv_cache_dtype: str = "auto"
    host: str = "0.0.0.0"
    port: int = 8080
    extra: dict = field(default_factory=dict)

    def __post_init__(self):
        # the attention kernels index the paged cache with shifts / masks
        b = self.block_size
        if b < 16 or b > 256 or b & (b - 1):
            raise ValueError(f"block_size must be a power of two in [16, 256], got {b}")
        if self.kv_cache_dtype not in KV_CACHE_DTYPES:
            raise ValueError(f"kv_cache_dtype must be one of {sorted(KV_CACHE_DTYPES)}, got {self.kv_cache_dtype!r}")

    @property
    def kv_fp8(self) -> bool:
        return KV_CACHE_DTYPES[self.kv_cache_dtype] == "fp8"

    def replace(self, **kw) -> "EngineConfig":
        return dataclasses.replace(self, **kw)

    @property
    def model_name(self) -> str:
        return self.served_model_name or self.model
