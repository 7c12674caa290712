"""Integer weight-only checkpoints (hipserve/weights/int_quant.py) on CPU.

The reference's HF chart serves an AWQ-8bit export of Qwen3-VL-30B-A3B
(vllm-models/helm-chart/values.yaml:8-12, compressed-tensors ``pack-quantized``).
No such checkpoint is reachable offline, so the tests write both layouts
(compressed-tensors pack-quantized, AutoAWQ gemm) from random integers with the
documented packing, check bit-exact unpacking, and check that a quantised tiny
checkpoint serves the same greedy tokens as transformers running the dequantised
weights (parity against the real export is unpinned).
"""
import json

import pytest
import torch

from hipserve.weights import int_quant as iq


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [True, False])
def test_pack_quantized_roundtrip(bits, sym):
    g = torch.Generator().manual_seed(bits)
    N, K, G = 24, 96, 32
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    q = torch.randint(lo, hi + 1, (N, K), generator=g)
    scale = torch.rand(N, K // G, generator=g) + 0.1
    zp = None if sym else torch.randint(lo, hi + 1, (N, K // G), generator=g)
    packed = iq.pack_pack_quantized(q, bits)
    assert packed.dtype == torch.int32 and packed.shape == (N, K * bits // 32)
    zp_packed = None if zp is None else iq.pack_pack_quantized(zp.t().contiguous(), bits).t().contiguous()
    got = iq.dequant_pack_quantized(packed, scale, zp_packed, torch.tensor([N, K]), None)
    want = (q - (0 if zp is None else zp.repeat_interleave(G, 1))).float() * scale.repeat_interleave(G, 1)
    assert torch.equal(got, want)
    # unpacked zero points and bits-from-config give the same answer
    got2 = iq.dequant_pack_quantized(packed, scale, zp, None, bits)
    assert torch.equal(got2, want)


def test_awq_roundtrip_and_order():
    g = torch.Generator().manual_seed(0)
    K, N, G = 64, 32, 16
    q = torch.randint(0, 16, (K, N), generator=g)
    z = torch.randint(0, 16, (K // G, N), generator=g)
    s = torch.rand(K // G, N, generator=g).half()
    qw = iq.awq_pack(q)
    # AutoAWQ's interleave: nibble 1 of word 0 holds column 2
    assert int(qw[0, 0] >> 4 & 0xF) == int(q[0, 2])
    w = iq.dequant_awq(qw, iq.awq_pack(z), s)
    want = ((q - z.repeat_interleave(G, 0)).float() * s.float().repeat_interleave(G, 0)).t()
    assert w.shape == (N, K) and torch.equal(w, want)


transformers = pytest.importorskip("transformers")


def _quantise_ckpt(m, path, fmt, bits=8, group=32):
    """Rewrite the saved checkpoint with every decoder Linear weight group-quantised in
    ``fmt``; returns transformers' model of the dequantised weights (the reference)."""
    import shutil

    from safetensors.torch import load_file, save_file

    m.save_pretrained(str(path), safe_serialization=True)
    sd = {}
    for f in sorted(path.glob("*.safetensors")):
        sd.update(load_file(str(f)))
        f.unlink()
    out, ref = {}, dict(sd)
    for k, w in sd.items():
        if ".layers." not in k or not k.endswith("proj.weight") or w.dim() != 2:
            out[k] = w
            continue
        N, K = w.shape
        qmax = (1 << (bits - 1)) - 1
        base = k[: -len(".weight")]
        if fmt == "ct":
            scale = w.reshape(N, K // group, group).abs().amax(-1).clamp_min(1e-8) / qmax
            q = torch.round(w / scale.repeat_interleave(group, 1)).clamp(-qmax - 1, qmax).to(torch.int64)
            out[base + ".weight_packed"] = iq.pack_pack_quantized(q, bits)
            out[base + ".weight_scale"] = scale.to(torch.bfloat16)
            out[base + ".weight_shape"] = torch.tensor([N, K], dtype=torch.int32)
            deq = iq.dequant_pack_quantized(out[base + ".weight_packed"], out[base + ".weight_scale"],
                                            None, out[base + ".weight_shape"], None)
        else:  # AutoAWQ 4-bit, asymmetric
            wt = w.t().reshape(K // group, group, N)
            lo, hi = wt.amin(1), wt.amax(1)
            s = ((hi - lo).clamp_min(1e-8) / 15).half()
            z = torch.round(-lo / s.float()).clamp(0, 15)
            q = torch.round(w.t() / s.float().repeat_interleave(group, 0) + z.repeat_interleave(group, 0))
            q = q.clamp(0, 15).to(torch.int64)
            out[base + ".qweight"] = iq.awq_pack(q)
            out[base + ".qzeros"] = iq.awq_pack(z.to(torch.int64))
            out[base + ".scales"] = s
            deq = iq.dequant_awq(out[base + ".qweight"], out[base + ".qzeros"], s)
        ref[k] = deq.to(w.dtype)
    refdir = path.parent / (path.name + "-ref")
    shutil.copytree(path, refdir)
    save_file(ref, str(refdir / "model.safetensors"))
    save_file(out, str(path / "model.safetensors"))
    cfg = json.loads((path / "config.json").read_text())
    cfg["quantization_config"] = (
        {"quant_method": "compressed-tensors", "format": "pack-quantized",
         "config_groups": {"group_0": {"targets": ["Linear"], "weights": {
             "num_bits": bits, "group_size": group, "symmetric": True, "strategy": "group", "type": "int"}}},
         "ignore": ["lm_head"]} if fmt == "ct" else
        {"quant_method": "awq", "bits": 4, "group_size": group, "version": "gemm", "zero_point": True})
    (path / "config.json").write_text(json.dumps(cfg))
    return transformers.AutoModelForCausalLM.from_pretrained(str(refdir), dtype=torch.float32).eval()


@pytest.mark.parametrize("fmt,family", [("ct", "qwen3_moe"), ("ct", "llama"), ("awq", "llama")])
def test_quantised_checkpoint_serves_dequantised_model(tmp_path, fmt, family):
    from hipserve.config import EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.parallel.comm import TPGroup

    common = dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                  vocab_size=320, max_position_embeddings=512, rms_norm_eps=1e-6, tie_word_embeddings=False)
    if family == "llama":
        cfg = transformers.LlamaConfig(**common, intermediate_size=128, head_dim=16)
    else:
        cfg = transformers.Qwen3MoeConfig(**common, intermediate_size=128, moe_intermediate_size=64,
                                          num_experts=4, num_experts_per_tok=2, norm_topk_prob=True,
                                          head_dim=16)
    torch.manual_seed(7)
    m = transformers.AutoModelForCausalLM.from_config(cfg, dtype=torch.float32).eval()
    if family == "qwen3_moe":
        with torch.no_grad():
            for n, p in m.named_parameters():
                if n.endswith("gate.weight"):
                    p.mul_(20.0)  # decisive routing
    path = tmp_path / f"{family}-{fmt}"
    m = _quantise_ckpt(m, path, fmt, bits=8 if fmt == "ct" else 4)
    eng = LLMEngine(EngineConfig(model=str(path), device="cpu", dtype="float32", max_num_seqs=2,
                                 max_num_batched_tokens=32, num_kv_blocks=64, max_model_len=128),
                    tp=TPGroup())
    prompts = [[1, 5, 9, 33, 70, 100], list(range(3, 30))]
    res = eng.generate(prompts, SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True))
    for p, (toks, _, _) in zip(prompts, res):
        with torch.no_grad():
            lg = m(torch.tensor([list(p) + list(toks)])).logits[0].float()
        for i, t in enumerate(toks):
            row = lg[len(p) - 1 + i]
            assert row[t] >= row.max() - 1e-4, (fmt, family, i, t, int(row.argmax()))
