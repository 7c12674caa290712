"""Qwen3-VL vision tower on the GPU (csrc/kernels/vision.hip) vs plain-PyTorch fp32
references: LayerNorm (+ fused residual add), GELU (tanh / erf), 2D RoPE + per-frame
bidirectional attention (head_dim 72 as in the Qwen3-VL-30B/235B towers, 64, 128;
ragged segments incl. partial last tiles), the whole bf16 tower vs the fp32 CPU tower
on the same checkpoint, and the bf16 engine's greedy tokens on an image prompt vs the
fp32 CPU engine."""
import numpy as np
import pytest
import torch

from hipserve.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from hipserve.ops import KernelOps

    return KernelOps()


@pytest.mark.parametrize("rows,C", [(37, 1152), (300, 4608), (5, 64), (64, 1280)])
@pytest.mark.parametrize("add", [False, True])
def test_layernorm_vs_fp32(ops, rows, C, add):
    torch.manual_seed(rows + C)
    x = (torch.randn(rows, C, device=DEV) * 2 + 0.5).bfloat16()
    w = (1 + 0.1 * torch.randn(C, device=DEV)).bfloat16()
    b = (0.1 * torch.randn(C, device=DEV)).bfloat16()
    r = torch.randn(rows, C, device=DEV).bfloat16() if add else None
    out = torch.empty_like(x)
    r_in = r.clone() if add else None
    ops.layernorm(out, x, w, b, 1e-6, residual=r_in)
    if add:
        want, rr = ref.add_layernorm(x, r, w, b, 1e-6)
        assert torch.equal(r_in, rr)
    else:
        want = ref.layernorm(x, w, b, 1e-6)
    assert (out.float() - want.float()).abs().max() <= 0.02 * want.float().abs().max()


@pytest.mark.parametrize("tanh", [True, False])
def test_gelu_vs_fp32(ops, tanh):
    x = (torch.randn(1000, 4304, device=DEV) * 3).bfloat16()
    want = ref.gelu(x, tanh)
    ops.gelu_(x, tanh)
    assert (x.float() - want.float()).abs().max() <= 1e-2


def _geo(lens):
    from hipserve.models.vision import ImageGeometry

    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    return ImageGeometry([], None, None, None, cu)


@pytest.mark.parametrize("D,nh,lens", [(72, 16, [1024, 96, 333]), (64, 16, [64, 700]), (128, 4, [130, 257]),
                                       (72, 2, [16])])
def test_vision_attention_vs_fp32(ops, D, nh, lens):
    torch.manual_seed(D + nh)
    T = sum(lens)
    qkv = (torch.randn(T, 3 * nh * D, device=DEV)).bfloat16()
    pos = torch.randint(0, 64, (T, 2))
    from hipserve.models.vision import rope_table_2d

    cs = rope_table_2d(pos, D).to(DEV)
    geo = _geo(lens)
    meta = ops.vision_meta(geo, nh, D)
    q_ref = qkv.clone()
    ref.vision_rope(q_ref, cs, nh, D)
    want = ref.vision_attention(q_ref, geo.cu_seqlens, nh, D, D ** -0.5).float()
    out = torch.empty(T, nh * D, device=DEV, dtype=torch.bfloat16)
    q_k = qkv.clone()
    ops.vision_attention(out, q_k, cs, meta[0], nh, D, D ** -0.5, meta)
    torch.cuda.synchronize()
    # rotated q/k: within one bf16 rounding of the fp32 reference (the kernel uses FMAs)
    a, b = q_k[:, : 2 * nh * D].float(), q_ref[:, : 2 * nh * D].float()
    assert ((a - b).abs() <= 2 ** -7 * b.abs() + 1e-6).all()
    err = (out.float() - want).abs().max().item()
    assert err <= 2e-2 * want.abs().max().item() + 1e-3, err


def test_vision_tower_and_engine_gpu_vs_cpu(tmp_path):
    transformers = pytest.importorskip("transformers")
    pytest.importorskip("PIL")
    from hipserve.config import EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.models.vision import image_geometry
    from hipserve.multimodal import MultiModalPrompt, expand_image_tokens, preprocess_image
    from hipserve.parallel.comm import TPGroup

    T = transformers
    tc = dict(hidden_size=256, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2, head_dim=64,
              intermediate_size=512, vocab_size=1024, max_position_embeddings=4096, rms_norm_eps=1e-6,
              rope_parameters={"rope_type": "default", "rope_theta": 1e6, "mrope_section": [12, 10, 10],
                               "mrope_interleaved": True})
    vc = dict(depth=3, hidden_size=144, intermediate_size=320, num_heads=2, patch_size=16, temporal_patch_size=2,
              in_channels=3, spatial_merge_size=2, out_hidden_size=256, num_position_embeddings=64,
              deepstack_visual_indexes=[1], hidden_act="gelu_pytorch_tanh")
    cfg = T.Qwen3VLConfig(text_config=tc, vision_config=vc, image_token_id=900, video_token_id=901,
                          vision_start_token_id=902, vision_end_token_id=903, tie_word_embeddings=False)
    torch.manual_seed(3)
    m = T.Qwen3VLForConditionalGeneration(cfg).eval()
    with torch.no_grad():
        for _, p in m.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.1)
    m.save_pretrained(str(tmp_path), safe_serialization=True)

    def eng(device):
        dt = "bfloat16" if device == "cuda" else "float32"
        dev = torch.device(device, 0) if device == "cuda" else torch.device("cpu")
        return LLMEngine(EngineConfig(model=str(tmp_path), device=device, dtype=dt, max_num_seqs=4,
                                      max_num_batched_tokens=512, max_model_len=2048, num_kv_blocks=256),
                         tp=TPGroup(0, 1, None, dev))

    g, c = eng("cuda"), eng("cpu")
    import dataclasses

    import PIL.Image

    vcfg = dataclasses.replace(g.model_cfg.vision, min_pixels=64 * 64, max_pixels=320 * 320)
    rng = np.random.default_rng(0)
    ims = [preprocess_image(PIL.Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)), vcfg)
           for w, h in ((300, 200), (160, 256))]
    pix = np.concatenate([i.pixels for i in ims])
    geo = image_geometry([i.grid for i in ims], vcfg)
    eg, dg = g.runner.model.visual.forward(torch.from_numpy(pix), geo)
    ec, dc = c.runner.model.visual.forward(torch.from_numpy(pix), geo)
    for a, b in [(eg, ec)] + list(zip(dg, dc)):
        rel = (a.float().cpu() - b).norm() / b.norm()
        assert rel < 0.03, rel
    ids = expand_image_tokens([1, 5, 902, 900, 903, 7, 8, 902, 900, 903, 9], ims, vcfg)
    sp = SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True)
    rg = g.generate([MultiModalPrompt(ids, ims)], sp)
    rc = c.generate([MultiModalPrompt(ids, ims)], sp)
    assert rg[0][0][0] == rc[0][0][0]  # first greedy token (bf16 vs fp32 engines)
