"""Quantised MoE experts on the GPU (gguf_mfma.hip MoE mode, ``qmoe_gemm``): INT8
(compressed-tensors 8-bit, the reference's Qwen3-VL-30B-A3B AWQ-8bit export) and
per-channel FP8 experts, against an fp32 reference of the same routed computation on
the dequantised weights; graph capture; and a per-expert INT8 checkpoint served
natively vs the same checkpoint dequantised to bf16 at load."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _qmoe(w, kind, kmajor=False):
    from hipserve.ops import quant as Q

    parts, deq = [], []
    for e in range(w.shape[0]):
        wf = w[e].float()
        if kind == "int8":
            s = wf.abs().amax(1, keepdim=True).clamp_min(1e-12) / 127.0
            q = torch.round(wf / s).clamp(-127, 127)
            parts.append(Q.QuantPart.from_int8((q + 128).to(torch.uint8), s, None, DEV))
            deq.append(q * s)
        else:
            s = wf.abs().amax(1, keepdim=True).clamp_min(1e-12) / 448.0
            q = (wf / s).to(torch.float8_e4m3fn)
            parts.append(Q.QuantPart.from_fp8(q, s, DEV))
            deq.append(q.float() * s)
    return Q.QuantMoE(parts, kmajor=kmajor), torch.stack(deq)


@pytest.mark.parametrize("kind", ["int8", "fp8"])
@pytest.mark.parametrize("T,E,k,I", [(6, 8, 2, 768), (40, 8, 2, 512), (200, 8, 2, 512), (33, 64, 4, 256)])
def test_quant_moe_vs_fp32(kind, T, E, k, I):
    from hipserve.config import PRESETS
    from hipserve.models.llama import LayerWeights, LlamaModel
    from hipserve.ops import KernelOps
    from hipserve.parallel.comm import TPGroup

    H = 512
    cfg = PRESETS["tiny-mixtral"].replace(hidden_size=H, intermediate_size=I, num_experts=E, num_experts_per_tok=k)
    m = LlamaModel(cfg, TPGroup(0, 1, None, torch.device(DEV)), DEV, torch.bfloat16, KernelOps())
    torch.manual_seed(T + E + I)
    router = torch.randn(E, H, device=DEV, dtype=torch.bfloat16) * 0.3
    w13, d13 = _qmoe(torch.randn(E, 2 * I, H, device=DEV) * 0.05, kind, kmajor=True)
    w2, d2 = _qmoe(torch.randn(E, H, I, device=DEV) * 0.05, kind)
    lw = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None, router=router, w13=w13, w2=w2)
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    got = m.moe(x, lw).float()
    logits = torch.nn.functional.linear(x, router).float()
    wts, idx = torch.topk(torch.softmax(logits, -1), k, -1)
    wts = wts / wts.sum(-1, keepdim=True)
    want = torch.zeros(T, H, device=DEV)
    xf = x.float()
    for e in range(E):
        rows, slot = (idx == e).nonzero(as_tuple=True)
        if rows.numel() == 0:
            continue
        gu = xf[rows] @ d13[e].T
        act = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
        want.index_add_(0, rows, (act @ d2[e].T) * wts[rows, slot].unsqueeze(-1))
    err = (got - want).abs().max().item()
    assert err <= 3e-2 * want.abs().max().item() + 1e-3, err
    # prefill-sized batches take the bf16 experts (dequantised scratch) and agree too
    from hipserve.ops import quant as Q

    assert torch.equal(Q.moe_dense(w13, 0), d13.to(torch.bfloat16)) or \
        (Q.moe_dense(w13, 0).float() - d13).abs().max().item() <= 1e-2 * d13.abs().max().item()
    # the decode path is device-only: capturable in a hipGraph
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        m.moe(x, lw)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out_g = m.moe(x, lw)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(out_g.float(), got)


def _per_expert_int8_ckpt(path, group=32):
    """Tiny Qwen3-MoE written like an llm-compressor export: per-expert gate/up/down
    Linear weights as compressed-tensors pack-quantized 8-bit (group scales)."""
    import json

    import transformers
    from safetensors.torch import load_file, save_file

    from hipserve.weights import int_quant as iq

    cfg = transformers.Qwen3MoeConfig(hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                                      num_key_value_heads=2, head_dim=64, intermediate_size=512,
                                      moe_intermediate_size=256, num_experts=16, num_experts_per_tok=4,
                                      norm_topk_prob=True, vocab_size=320, max_position_embeddings=512,
                                      rms_norm_eps=1e-6, tie_word_embeddings=False)
    torch.manual_seed(5)
    m = transformers.AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).eval()
    with torch.no_grad():
        for name, p in m.named_parameters():
            if name.endswith("gate.weight"):
                p.mul_(20.0)
    m.save_pretrained(str(path), safe_serialization=True)
    sd = {}
    for f in sorted(path.glob("*.safetensors")):
        sd.update(load_file(str(f)))
        f.unlink()
    out = {}

    def q8(base, w):
        N, K = w.shape
        scale = w.reshape(N, K // group, group).abs().amax(-1).clamp_min(1e-8) / 127
        q = torch.round(w / scale.repeat_interleave(group, 1)).clamp(-128, 127).to(torch.int64)
        out[base + ".weight_packed"] = iq.pack_pack_quantized(q, 8)
        out[base + ".weight_scale"] = scale.to(torch.bfloat16)
        out[base + ".weight_shape"] = torch.tensor([N, K], dtype=torch.int32)

    I = cfg.moe_intermediate_size
    for k, w in sd.items():
        if ".experts." in k and k.endswith("_proj.weight") and w.dim() == 2:  # per-expert export
            q8(k[: -len(".weight")], w)
        elif k.endswith("experts.gate_up_proj"):  # fused layout (older/newer exports)
            base = k[: -len("gate_up_proj")]
            for e in range(w.shape[0]):
                q8(f"{base}{e}.gate_proj", w[e, :I])
                q8(f"{base}{e}.up_proj", w[e, I:])
        elif k.endswith("experts.down_proj"):
            base = k[: -len("down_proj")]
            for e in range(w.shape[0]):
                q8(f"{base}{e}.down_proj", w[e])
        else:
            out[k] = w
    save_file(out, str(path / "model.safetensors"))
    c = json.loads((path / "config.json").read_text())
    c["quantization_config"] = {"quant_method": "compressed-tensors", "format": "pack-quantized",
                                "config_groups": {"group_0": {"targets": ["Linear"], "weights": {
                                    "num_bits": 8, "group_size": group, "symmetric": True, "strategy": "group",
                                    "type": "int"}}}, "ignore": ["lm_head"]}
    (path / "config.json").write_text(json.dumps(c))


def test_int8_expert_checkpoint_native(tmp_path):
    pytest.importorskip("transformers")
    import hipserve.models.llama as L
    from hipserve.config import EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.ops import quant as Q
    from hipserve.parallel.comm import TPGroup

    path = tmp_path / "qwen3moe-int8"
    _per_expert_int8_ckpt(path)
    prompts = [[1, 5, 9, 33, 70, 100], list(range(3, 40)), [7] * 12]
    got = {}
    for native in (True, False):
        L.LlamaModel.native_fp8 = native
        try:
            eng = LLMEngine(EngineConfig(model=str(path), device="cuda", max_num_seqs=4, max_num_batched_tokens=128,
                                         num_kv_blocks=64, max_model_len=256),
                            tp=TPGroup(0, 1, None, torch.device("cuda", 0)))
        finally:
            L.LlamaModel.native_fp8 = True
        mm = eng.runner.model
        assert isinstance(mm.layers[0].w13, Q.QuantMoE) == native
        orig = mm.compute_logits

        def cap(h, orig=orig, native=native):
            out = orig(h)
            got.setdefault(native, []).append(out.float().cpu().clone())
            return out

        mm.compute_logits = cap
        eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True))
        eng.shutdown()
    a, b = torch.cat(got[True]), torch.cat(got[False])
    assert a.shape == b.shape
    assert (a - b).abs().max().item() < 5e-2 * b.abs().max().item() + 1e-3
    assert (a.argmax(-1) == b.argmax(-1)).float().mean().item() >= 0.85


@pytest.mark.parametrize("kind", ["int8", "fp8"])
@pytest.mark.parametrize("packed", [False, True])
def test_quant_moe_prefill_paths_vs_fp32(kind, packed):
    """Prefill-sized routing of quantised experts: the row-major dequantised scratch with
    the weight-streaming expert kernel (``MOE_PACKED_PREFILL = "0"``), and the dequantised
    + packed scratch with the one-launch packed grouped GEMM (``"1"``), both against the
    fp32 reference."""
    from hipserve.config import PRESETS
    from hipserve.models import llama as L
    from hipserve.models.llama import LayerWeights, LlamaModel
    from hipserve.ops import KernelOps
    from hipserve.ops import quant as Q
    from hipserve.parallel.comm import TPGroup

    H, I, E, k = 512, 512, 16, 4
    T = L.MOE_KERNEL_MAX_PAIRS // k + 300
    cfg = PRESETS["tiny-mixtral"].replace(hidden_size=H, intermediate_size=I, num_experts=E, num_experts_per_tok=k)
    m = LlamaModel(cfg, TPGroup(0, 1, None, torch.device(DEV)), DEV, torch.bfloat16, KernelOps())
    m.MOE_PACKED_PREFILL = "1" if packed else "0"
    torch.manual_seed(7)
    router = torch.randn(E, H, device=DEV, dtype=torch.bfloat16) * 0.3
    w13, d13 = _qmoe(torch.randn(E, 2 * I, H, device=DEV) * 0.05, kind, kmajor=True)
    w2, d2 = _qmoe(torch.randn(E, H, I, device=DEV) * 0.05, kind)
    lw = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None, router=router, w13=w13, w2=w2)
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    got = m.moe(x, lw).float()
    logits = torch.nn.functional.linear(x, router).float()
    wts, idx = torch.topk(torch.softmax(logits, -1), k, -1)
    wts = wts / wts.sum(-1, keepdim=True)
    want = torch.zeros(T, H, device=DEV)
    xf = x.float()
    for e in range(E):
        rows, slot = (idx == e).nonzero(as_tuple=True)
        if rows.numel() == 0:
            continue
        gu = xf[rows] @ d13[e].T
        act = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
        want.index_add_(0, rows, (act @ d2[e].T) * wts[rows, slot].unsqueeze(-1))
    err = (got - want).abs().max().item()
    assert err <= 3e-2 * want.abs().max().item() + 1e-3, err
    if packed:  # the packed dequant equals packing the row-major dequant, bit for bit
        from hipserve.ops import gemm

        p13 = Q.moe_packed_scratch(w13, 0, True).clone()
        p2 = Q.moe_packed_scratch(w2, 1, False).clone()
        d13r, d2r = Q.moe_dense(w13, 0), Q.moe_dense(w2, 1)
        for e in range(E):
            assert torch.equal(p13[e], gemm.pack(d13r[e].contiguous(), glu=True))
            assert torch.equal(p2[e], gemm.pack(d2r[e].contiguous()))


@pytest.mark.parametrize("kind", ["int8", "int8g", "fp8"])
@pytest.mark.parametrize("T,E,k", [(5, 16, 4), (48, 16, 4), (64, 128, 8)])
def test_qmoe_glu_epilogue_and_kmajor_bit_exact(kind, T, E, k):
    """The w13 expert GEMM with the SiLU-GLU in its epilogue == the bf16 gate|up output
    then silu_and_mul, bit for bit; and super-chunk-major (k-major) expert weights give
    the same bits as the row-group-major layout (the same sums in the same order)."""
    from hipserve.ops import quant as Q

    op = torch.ops.hipserve
    H, I = 512, 768
    torch.manual_seed(T + E)
    parts = []
    for _ in range(E):
        wf = torch.randn(2 * I, H, device=DEV) * 0.05
        if kind == "fp8":
            s = wf.abs().amax(1, keepdim=True) / 448.0
            parts.append(Q.QuantPart.from_fp8((wf / s).to(torch.float8_e4m3fn), s, DEV))
        else:
            G = 32 if kind == "int8g" else H
            s = wf.view(2 * I, H // G, G).abs().amax(-1) / 127.0
            q = torch.round(wf / s.repeat_interleave(G, 1)).clamp(-127, 127)
            parts.append(Q.QuantPart.from_int8((q + 128).to(torch.uint8), s, None, DEV))
    w = Q.QuantMoE(parts)
    assert w.kqt == {"fp8": 6, "int8": 9, "int8g": 8}[kind]
    P = T * k
    tile = 16 if P <= 8 * E else 32
    cap = -(-(P + E * (tile - 1)) // tile) * tile
    ids = torch.topk(torch.rand(T, E, device=DEV), k, dim=-1).indices.int()
    slots = torch.empty(cap, dtype=torch.int32, device=DEV)
    te = torch.empty(cap // tile, dtype=torch.int32, device=DEV)
    nt = torch.empty(1, dtype=torch.int32, device=DEV)
    ps = torch.empty(P, dtype=torch.int32, device=DEV)
    op.moe_align(ids, E, tile, slots, te, nt, ps)
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    f32 = torch.empty(0, dtype=torch.float32, device=DEV)
    gu = torch.zeros(cap, 2 * I, device=DEV, dtype=torch.bfloat16)
    op.qmoe_gemm(gu, f32, x, w.q, w.rs, w.kqt, w.N, w.K, slots, te, tile, k, 1)
    want = torch.zeros(cap, I, device=DEV, dtype=torch.bfloat16)
    torch.ops.hipserve.silu_and_mul(want, gu)
    real = slots >= 0
    G, nsb = w.N // 16, w.K // 256
    qk = w.q.view(w.E, G, nsb, -1).transpose(1, 2).contiguous().view(w.E, -1)
    for q, km in ((w.q, False), (qk, True)):
        act = torch.zeros(cap, I, device=DEV, dtype=torch.bfloat16)
        op.qmoe_gemm(act, f32, x, q, w.rs, w.kqt, w.N, w.K, slots, te, tile, k, 1, km, 1)
        assert torch.equal(act[real], want[real]), km
        gk = torch.zeros_like(gu)
        op.qmoe_gemm(gk, f32, x, q, w.rs, w.kqt, w.N, w.K, slots, te, tile, k, 1, km)
        assert torch.equal(gk[real], gu[real]), km
