"""Model families end to end on the GPU (HIP kernels, hipGraph decode): a tiny HF
checkpoint per family (written by ``transformers`` on the CPU) served by the bf16
GPU engine must agree with the fp32 CPU reference engine loading the same files
(first greedy token; graph vs eager decode). Shapes are chosen so the GPU-only
paths run: per-head q/k RMSNorm kernel (Qwen3, Gemma-3), qkv bias (Qwen2), the MoE
decode kernels with 16 experts and renormalised top-4 (Qwen3-MoE), GeGLU + sandwich
norms + sliding-window prefill/decode attention + local RoPE (Gemma-3, head_dim
128 -> prefill v2), head_dim 96 attention (Phi-3)."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from hipserve.config import EngineConfig  # noqa: E402
from hipserve.engine.llm_engine import LLMEngine  # noqa: E402
from hipserve.engine.request import SamplingParams  # noqa: E402
from hipserve.parallel.comm import TPGroup  # noqa: E402

pytestmark = pytest.mark.gpu

BASE = dict(hidden_size=256, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, vocab_size=1024,
            max_position_embeddings=4096, rms_norm_eps=1e-6, tie_word_embeddings=False)


def _cfg(family):
    T = transformers
    return {
        "qwen2": lambda: T.Qwen2Config(**BASE, intermediate_size=512, rope_theta=1e6),
        "qwen3": lambda: T.Qwen3Config(**BASE, intermediate_size=512, head_dim=64, rope_theta=1e6),
        "qwen3_moe": lambda: T.Qwen3MoeConfig(**BASE, intermediate_size=512, moe_intermediate_size=256,
                                              num_experts=16, num_experts_per_tok=4, norm_topk_prob=True,
                                              head_dim=64, rope_theta=1e6),
        "gemma3": lambda: T.Gemma3TextConfig(
            **{**BASE, "num_hidden_layers": 3, "tie_word_embeddings": True}, intermediate_size=512, head_dim=128,
            query_pre_attn_scalar=64, sliding_window=64,
            rope_parameters={"sliding_attention": {"rope_type": "default", "rope_theta": 1e4},
                             "full_attention": {"rope_type": "linear", "factor": 2.0, "rope_theta": 1e6}},
            layer_types=["sliding_attention", "sliding_attention", "full_attention"]),
        "phi3": lambda: T.Phi3Config(**{**BASE, "hidden_size": 384, "num_key_value_heads": 4},
                                     intermediate_size=512, rope_theta=10000.0, pad_token_id=0),
    }[family]()


PROMPTS = [[1] + list(range(10, 300)), [1, 7, 8, 9], [1] + [42] * 40, list(range(3, 600))]


@pytest.fixture(scope="module")
def ckpts(tmp_path_factory):
    out = {}
    for fam in ("qwen2", "qwen3", "qwen3_moe", "gemma3", "phi3"):
        torch.manual_seed(7)
        m = transformers.AutoModelForCausalLM.from_config(_cfg(fam), torch_dtype=torch.float32)
        with torch.no_grad():
            for name, p in m.named_parameters():
                if p.dim() == 1:
                    p.add_(torch.randn_like(p) * 0.1)
                elif name.endswith("gate.weight") and p.shape[0] == 16:
                    p.mul_(20.0)  # decisive routing
        path = tmp_path_factory.mktemp(fam)
        m.save_pretrained(str(path), safe_serialization=True)
        out[fam] = str(path)
    return out


def _engine(path, device, eager):
    dt = "bfloat16" if device == "cuda" else "float32"
    cfg = EngineConfig(model=path, device=device, dtype=dt, max_num_seqs=16, max_num_batched_tokens=256,
                       max_model_len=2048, num_kv_blocks=512, enforce_eager=eager)
    dev = torch.device(device, 0) if device == "cuda" else torch.device("cpu")
    return LLMEngine(cfg, tp=TPGroup(0, 1, None, dev))


@pytest.mark.parametrize("family", ["qwen2", "qwen3", "qwen3_moe", "gemma3", "phi3"])
def test_family_gpu_matches_cpu(ckpts, family):
    sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    g = _engine(ckpts[family], "cuda", eager=False)
    assert g.runner.use_graphs and g.runner.graphs
    e = _engine(ckpts[family], "cuda", eager=True)
    c = _engine(ckpts[family], "cpu", eager=True)
    rg, re_, rc = g.generate(PROMPTS, sp), e.generate(PROMPTS, sp), c.generate(PROMPTS, sp)
    for a, b in zip(rg, re_):
        assert len(a[0]) == 6 and a[0][:2] == b[0][:2], (family, rg, re_)
    first = sum(a[0][0] == b[0][0] for a, b in zip(rg, rc))
    assert first >= len(PROMPTS) - 1, (family, rg, rc)
