"""Which decode layers take the fused qkv-partials -> RoPE + KV write + attention kernel
(attention_decode.hip QkvIn, ``LlamaModel.fused_qkv_attn_ok``) and how the qkv decode GEMM
is tuned for it (``fused_gemm_shapes``): a pure policy test, no kernels run."""
import torch

from hipserve.config import PRESETS
from hipserve.models.llama import LlamaModel
from hipserve.ops import get_ops
from hipserve.parallel.comm import TPGroup


def _model(**kw):
    cfg = PRESETS["llama-3-8b"].replace(hidden_size=256, intermediate_size=768, num_heads=4, num_kv_heads=2,
                                        num_layers=3, vocab_size=512, max_position_embeddings=512, **kw)
    m = LlamaModel(cfg, TPGroup(0, 1, None, torch.device("cpu")), "cpu", torch.bfloat16, get_ops("cpu"),
                   max_pos=512)
    m.allocate_random(seed=0)
    return m


def test_llama_bf16_cache_fused_everywhere():
    m = _model()
    assert m.fused_qkv_attention  # the default (HIPSERVE_FUSED_QKV_ATTN unset)
    assert m.fused_qkv_attn_ok() and all(m.fused_qkv_attn_ok(i) for i in range(3))
    if m.fused_family:
        spec = m.fused_gemm_shapes()[tuple(m.layers[0].wqkv.shape)]
        assert spec[0] == "attn"  # timed as the partial GEMM alone


def test_e4m3_cache_takes_the_separate_writer():
    m = _model()
    m.kv_dtype = torch.float8_e4m3fn
    assert not m.fused_qkv_attn_ok()
    if m.fused_family:
        assert m.fused_gemm_shapes()[tuple(m.layers[0].wqkv.shape)][0] == "rope"


def test_qk_norm_needs_rotate_half():
    m = _model(family="qwen3", qk_norm=True)
    assert m.layers[0].q_norm is not None
    assert m.fused_qkv_attn_ok() == (m.cfg.rope_mode == 0)
    m.cfg = m.cfg.replace(rope_mode=1)
    assert not m.fused_qkv_attn_ok()


def test_qkv_bias_and_sliding_window_layers_unfused():
    m = _model(family="qwen2", qkv_bias=True)
    assert not m.fused_qkv_attn_ok()
    g = _model(sliding_window=64, layer_windows=(64, 0, 64))
    assert [g.fused_qkv_attn_ok(i) for i in range(3)] == [False, True, False]
    assert not g.fused_qkv_attn_ok()  # not on every layer: the tuner keeps the RoPE unit


def test_opt_out():
    m = _model()
    m.fused_qkv_attention = False
    assert not m.fused_qkv_attn_ok()
