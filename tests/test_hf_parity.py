"""Model-family parity against HuggingFace ``transformers`` on CPU.

A tiny random checkpoint of each served architecture is written with
``save_pretrained`` (safetensors + config.json: what an HF-tier PVC holds), loaded
by hipserve's safetensors loader, and the engine's greedy continuation (paged KV,
chunked prefill, batched decode, reference ops) must be the argmax of the
transformers forward at every step (teacher-forced, fp32).

Families: Llama, Mixtral, Qwen2 (qkv bias), Qwen3 (per-head q/k RMSNorm),
Qwen3-MoE (top-k renormalisation on / off), Gemma-3 text (GeGLU, sandwich norms,
embedding scale, sliding-window layers with their own RoPE base, linear RoPE
scaling on the global layers) and Phi-3 (fused qkv / gate_up tensors). The
reference's chart defaults (vllm-models/helm-chart/values.yaml:1-19: Gemma-3-27B,
Qwen3-VL-30B-A3B, Qwen3-0.6B; ramalama-models/helm-chart/values.yaml:3-19:
TinyLlama, Phi-3-mini) are these families' text models.
"""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from hipserve.config import EngineConfig  # noqa: E402
from hipserve.engine.llm_engine import LLMEngine  # noqa: E402
from hipserve.engine.request import SamplingParams  # noqa: E402
from hipserve.parallel.comm import TPGroup  # noqa: E402

COMMON = dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
              vocab_size=320, max_position_embeddings=512, rms_norm_eps=1e-6, tie_word_embeddings=False)


def _configs():
    T = transformers
    return {
        "llama": lambda: T.LlamaConfig(**COMMON, intermediate_size=128, rope_theta=10000.0, head_dim=16),
        "mixtral": lambda: T.MixtralConfig(**COMMON, intermediate_size=96, rope_theta=1e6, num_local_experts=4,
                                           num_experts_per_tok=2),
        "qwen2": lambda: T.Qwen2Config(**COMMON, intermediate_size=128, rope_theta=1e6),
        "qwen3": lambda: T.Qwen3Config(**COMMON, intermediate_size=128, rope_theta=1e6, head_dim=32),
        "qwen3_moe": lambda: T.Qwen3MoeConfig(**COMMON, intermediate_size=128, moe_intermediate_size=48,
                                              num_experts=8, num_experts_per_tok=3, norm_topk_prob=True,
                                              head_dim=16, rope_theta=1e6),
        "qwen3_moe_nonorm": lambda: T.Qwen3MoeConfig(**COMMON, intermediate_size=128, moe_intermediate_size=48,
                                                     num_experts=8, num_experts_per_tok=2, norm_topk_prob=False,
                                                     head_dim=16, rope_theta=1e6),
        "gemma3": lambda: T.Gemma3TextConfig(
            **{**COMMON, "num_hidden_layers": 3, "tie_word_embeddings": True}, intermediate_size=128,
            head_dim=32, query_pre_attn_scalar=24, sliding_window=8,
            rope_parameters={"sliding_attention": {"rope_type": "default", "rope_theta": 1e4},
                             "full_attention": {"rope_type": "linear", "factor": 2.0, "rope_theta": 1e6}},
            layer_types=["sliding_attention", "sliding_attention", "full_attention"]),
        "phi3": lambda: T.Phi3Config(**{**COMMON, "num_key_value_heads": 4}, intermediate_size=128,
                                     rope_theta=10000.0, pad_token_id=0),
    }


def _build(tmp_path, family):
    cfg = _configs()[family]()
    torch.manual_seed(1234)
    m = transformers.AutoModelForCausalLM.from_config(cfg, torch_dtype=torch.float32).eval()
    with torch.no_grad():
        for name, p in m.named_parameters():
            if p.dim() == 1:  # non-trivial norm weights / biases (HF initialises them to 1 or 0)
                p.add_(torch.randn_like(p) * 0.1)
            elif name.endswith("gate.weight") and p.shape[0] <= 8:
                p.mul_(20.0)  # decisive MoE routing: no near-ties between experts
    path = tmp_path / family
    m.save_pretrained(str(path), safe_serialization=True)
    return m, str(path)


@pytest.mark.parametrize("family", list(_configs()))
def test_greedy_matches_transformers(tmp_path, family):
    m, path = _build(tmp_path, family)
    eng = LLMEngine(EngineConfig(model=path, device="cpu", dtype="float32", max_num_seqs=4,
                                 max_num_batched_tokens=24, num_kv_blocks=128, max_model_len=256),
                    tp=TPGroup())
    mc = eng.runner.model.cfg
    assert mc.family == family.split("_nonorm")[0]
    prompts = [[1, 5, 9, 33, 70, 100], list(range(3, 40)), [7] * 11]
    sp = SamplingParams(temperature=0.0, max_tokens=8, ignore_eos=True)
    res = eng.generate(prompts, sp)
    for p, (toks, _, reason) in zip(prompts, res):
        assert reason == "length" and len(toks) == 8
        with torch.no_grad():
            lg = m(torch.tensor([list(p) + list(toks)])).logits[0].float()
        for i, t in enumerate(toks):
            row = lg[len(p) - 1 + i]
            assert row[t] >= row.max() - 1e-4, (family, i, t, int(row.argmax()), float(row.max() - row[t]))


def _hf_to_gguf(m, family, path):
    """Write the HF model's tensors as an F32 GGUF of llama.cpp's layout for
    ``family`` (phi3: fused attn_qkv and ffn_up = [gate; up]; qwen2: q/k/v biases;
    qwen3: attn_q_norm / attn_k_norm)."""
    import numpy as np

    from hipserve.weights import gguf as G

    c = m.config
    sd = {k: v.detach().float().numpy() for k, v in m.state_dict().items()}
    H, V, L = c.hidden_size, c.vocab_size, c.num_hidden_layers
    D = getattr(c, "head_dim", None) or H // c.num_attention_heads
    a = family
    toks = ["<unk>", "<s>", "</s>"] + [f"<0x{b:02X}>" for b in range(256)] + [f"▁w{i}" for i in range(V - 259)]
    md = {"general.architecture": a, "general.name": f"tiny-{a}", f"{a}.context_length": 512,
          f"{a}.embedding_length": H, f"{a}.block_count": L, f"{a}.feed_forward_length": c.intermediate_size,
          f"{a}.attention.head_count": c.num_attention_heads,
          f"{a}.attention.head_count_kv": c.num_key_value_heads, f"{a}.attention.key_length": D,
          f"{a}.rope.freq_base": float(c.rope_parameters["rope_theta"]), f"{a}.rope.dimension_count": D,
          f"{a}.attention.layer_norm_rms_epsilon": float(c.rms_norm_eps),
          "tokenizer.ggml.model": "llama", "tokenizer.ggml.tokens": toks,
          "tokenizer.ggml.scores": [float(-i) for i in range(len(toks))],
          "tokenizer.ggml.token_type": [3 if i < 3 else (6 if i < 259 else 1) for i in range(len(toks))],
          "tokenizer.ggml.bos_token_id": 1, "tokenizer.ggml.eos_token_id": 2}
    t = [("token_embd.weight", sd["model.embed_tokens.weight"], G.F32),
         ("output_norm.weight", sd["model.norm.weight"], G.F32), ("output.weight", sd["lm_head.weight"], G.F32)]
    for i in range(L):
        p, b = f"model.layers.{i}.", f"blk.{i}."
        t += [(b + "attn_norm.weight", sd[p + "input_layernorm.weight"], G.F32),
              (b + "ffn_norm.weight", sd[p + "post_attention_layernorm.weight"], G.F32),
              (b + "attn_output.weight", sd[p + "self_attn.o_proj.weight"], G.F32),
              (b + "ffn_down.weight", sd[p + "mlp.down_proj.weight"], G.F32)]
        if a == "phi3":
            t += [(b + "attn_qkv.weight", sd[p + "self_attn.qkv_proj.weight"], G.F32),
                  (b + "ffn_up.weight", sd[p + "mlp.gate_up_proj.weight"], G.F32)]
        else:
            t += [(b + f"attn_{x}.weight", sd[p + f"self_attn.{x}_proj.weight"], G.F32) for x in "qkv"]
            t += [(b + "ffn_gate.weight", sd[p + "mlp.gate_proj.weight"], G.F32),
                  (b + "ffn_up.weight", sd[p + "mlp.up_proj.weight"], G.F32)]
        if a == "qwen2":
            t += [(b + f"attn_{x}.bias", sd[p + f"self_attn.{x}_proj.bias"], G.F32) for x in "qkv"]
        if a == "qwen3":
            t += [(b + "attn_q_norm.weight", sd[p + "self_attn.q_norm.weight"], G.F32),
                  (b + "attn_k_norm.weight", sd[p + "self_attn.k_norm.weight"], G.F32)]
    G.write_gguf(path, md, [(n, np.ascontiguousarray(x), q) for n, x, q in t])
    return path


@pytest.mark.parametrize("family", ["phi3", "qwen2", "qwen3"])
def test_gguf_family_matches_transformers(tmp_path, family):
    """GGUF tier (llama-server role) for the non-llama llama.cpp architectures,
    incl. the reference's Phi-3-mini (ramalama-models/helm-chart/values.yaml:13-19):
    an F32 GGUF of the same weights greedy-decodes like transformers."""
    m, _ = _build(tmp_path, family)
    p = _hf_to_gguf(m, family, str(tmp_path / f"{family}.gguf"))
    eng = LLMEngine(EngineConfig(model=p, device="cpu", dtype="float32", load_format="gguf", max_num_seqs=4,
                                 max_num_batched_tokens=24, num_kv_blocks=128, max_model_len=256), tp=TPGroup())
    assert eng.runner.model.cfg.family == family and eng.runner.model.cfg.rope_mode == 0
    prompts = [[1, 5, 9, 33, 70, 100], list(range(3, 40))]
    res = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
    for pr, (toks, _, _) in zip(prompts, res):
        with torch.no_grad():
            lg = m(torch.tensor([list(pr) + list(toks)])).logits[0].float()
        for i, t in enumerate(toks):
            row = lg[len(pr) - 1 + i]
            assert row[t] >= row.max() - 1e-3, (family, i, t, int(row.argmax()))


def test_gemma3_hub_config_keys():
    """Hub-style Gemma-3 config.json (rope_theta / rope_local_base_freq / rope_scaling /
    sliding_window_pattern, multimodal text_config wrapper) maps to the same layout."""
    from hipserve.config import ModelConfig

    d = {"architectures": ["Gemma3ForConditionalGeneration"], "model_type": "gemma3",
         "text_config": {"model_type": "gemma3_text", "hidden_size": 5376, "num_hidden_layers": 62,
                         "num_attention_heads": 32, "num_key_value_heads": 16, "head_dim": 128,
                         "intermediate_size": 21504, "vocab_size": 262208, "query_pre_attn_scalar": 168,
                         "rope_theta": 1000000.0, "rope_local_base_freq": 10000.0,
                         "rope_scaling": {"rope_type": "linear", "factor": 8.0}, "sliding_window": 1024,
                         "sliding_window_pattern": 6, "rms_norm_eps": 1e-6},
         "eos_token_id": [1, 106]}
    c = ModelConfig.from_hf_dict(d)
    assert c.family == "gemma3" and c.rope_theta == 1e6 and c.rope_local_theta == 1e4
    assert c.rope_scaling["factor"] == 8.0 and c.sliding_window == 1024 and c.tie_word_embeddings
    assert c.layer_windows[:6] == (1024,) * 5 + (0,) and len(c.layer_windows) == 62
    assert abs(c.attn_scale - 168 ** -0.5) < 1e-12 and c.eos_token_id == (1, 106)


def test_qwen3_vl_moe_text_config():
    from hipserve.config import ModelConfig

    d = {"architectures": ["Qwen3VLMoeForConditionalGeneration"], "model_type": "qwen3_vl_moe",
         "text_config": {"model_type": "qwen3_vl_moe_text", "hidden_size": 2048, "num_hidden_layers": 48,
                         "num_attention_heads": 32, "num_key_value_heads": 4, "head_dim": 128,
                         "intermediate_size": 6144, "moe_intermediate_size": 768, "num_experts": 128,
                         "num_experts_per_tok": 8, "norm_topk_prob": True, "vocab_size": 151936,
                         "rope_theta": 5000000.0, "rms_norm_eps": 1e-6, "decoder_sparse_step": 1,
                         "mlp_only_layers": []}}
    c = ModelConfig.from_hf_dict(d)
    assert c.family == "qwen3_moe" and c.num_experts == 128 and c.expert_size == 768 and c.qk_norm


def test_fp8_checkpoint_dequantised_at_load(tmp_path):
    """compressed-tensors FP8 checkpoints (e.g. the reference's gemma-3-27b-it-FP8-Dynamic):
    float8 weights + per-channel weight_scale load as the dequantised weights."""
    from safetensors.torch import save_file

    from hipserve.weights.safetensors_loader import _Ckpt

    w = torch.randn(16, 32)
    scale = w.abs().amax(1, keepdim=True) / 448.0
    q = (w / scale).to(torch.float8_e4m3fn)
    save_file({"layer.weight": q, "layer.weight_scale": scale}, str(tmp_path / "model.safetensors"))
    ck = _Ckpt(str(tmp_path))
    got = ck.full("layer.weight")
    assert torch.allclose(got, q.float() * scale)
    assert torch.allclose(ck.rows("layer.weight", 4, 9), (q.float() * scale)[4:9])
    assert (got - w).abs().max() <= 0.07 * w.abs().max()
