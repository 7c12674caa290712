"""Qwen3-VL image input (the reference's default HF model family:
vllm-models/helm-chart/values.yaml:8-12) against HuggingFace ``transformers`` on CPU.

A tiny random Qwen3-VL checkpoint (``save_pretrained``: vision tower + language model)
is loaded by hipserve; pinned against transformers' Qwen3VLForConditionalGeneration:

* image preprocessing (smart resize, bicubic, normalise, 2x2-merge-block patch order)
  vs ``Qwen2VLImageProcessorPil`` with the Qwen3-VL settings;
* the vision tower (patch embedding, resampled position table, 2D RoPE, ViT
  blocks, DeepStack mergers, final merger) vs ``get_image_features``;
* MRoPE positions vs ``get_rope_index``;
* the engine's greedy continuation of a prompt holding two images (image
  embeddings spliced into prefill, DeepStack features added after the first
  decoder layers, interleaved MRoPE for image tokens, position delta afterwards,
  chunked prefill splitting an image) vs the teacher-forced transformers logits;
* the OpenAI chat surface: an ``image_url`` part is accepted for a vision model
  and rejected (400) for a text-only one; prefix caching never shares image KV
  between different images.
"""
import base64
import dataclasses
import io

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from hipserve.config import EngineConfig, ModelConfig, VisionConfig  # noqa: E402
from hipserve.engine.llm_engine import LLMEngine  # noqa: E402
from hipserve.engine.request import SamplingParams  # noqa: E402
from hipserve.multimodal import (MultiModalPrompt, expand_image_tokens, mm_state,  # noqa: E402
                                 preprocess_image)
from hipserve.parallel.comm import TPGroup  # noqa: E402

IMG, VS, VE = 300, 302, 303


def _hf_model(tmp_path, deepstack=(0, 1)):
    T = transformers
    tc = dict(hidden_size=64, num_hidden_layers=3, num_attention_heads=4, num_key_value_heads=2, head_dim=16,
              intermediate_size=128, vocab_size=400, max_position_embeddings=512, rms_norm_eps=1e-6,
              rope_parameters={"rope_type": "default", "rope_theta": 10000.0, "mrope_section": [2, 3, 3],
                               "mrope_interleaved": True})
    vc = dict(depth=3, hidden_size=32, intermediate_size=64, num_heads=2, patch_size=16, temporal_patch_size=2,
              in_channels=3, spatial_merge_size=2, out_hidden_size=64, num_position_embeddings=16,
              deepstack_visual_indexes=list(deepstack), hidden_act="gelu_pytorch_tanh")
    cfg = T.Qwen3VLConfig(text_config=tc, vision_config=vc, image_token_id=IMG, video_token_id=301,
                          vision_start_token_id=VS, vision_end_token_id=VE, tie_word_embeddings=False)
    torch.manual_seed(7)
    m = T.Qwen3VLForConditionalGeneration(cfg).eval()
    with torch.no_grad():
        for name, p in m.named_parameters():
            if p.dim() == 1:
                p.add_(torch.randn_like(p) * 0.1)
            else:
                p.mul_(3.0 if "visual" in name else 1.0)
    path = tmp_path / "tinyvl"
    m.save_pretrained(str(path), safe_serialization=True)
    return m, str(path)


def _vcfg(mc: ModelConfig) -> VisionConfig:
    return dataclasses.replace(mc.vision, min_pixels=32 * 32, max_pixels=128 * 128)


def _image(seed, w, h):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    return PIL.Image.fromarray(a)


def _hf_pixels(img, vc: VisionConfig):
    from transformers.models.qwen2_vl.image_processing_pil_qwen2_vl import Qwen2VLImageProcessorPil

    p = Qwen2VLImageProcessorPil(patch_size=16, merge_size=2, temporal_patch_size=2, image_mean=[0.5] * 3,
                                 image_std=[0.5] * 3, min_pixels=vc.min_pixels, max_pixels=vc.max_pixels)
    out = p(images=[img], return_tensors="np")
    return out["pixel_values"], out["image_grid_thw"]


def test_config_and_preprocessing(tmp_path):
    _, path = _hf_model(tmp_path)
    import json

    with open(f"{path}/config.json") as f:
        mc = ModelConfig.from_hf_dict(json.load(f))
    assert mc.family == "qwen3" and mc.mrope_section == (2, 3, 3) and mc.vision is not None
    assert mc.vision.deepstack_visual_indexes == (0, 1) and mc.vision.image_token_id == IMG
    vc = _vcfg(mc)
    for seed, (w, h) in enumerate([(70, 45), (128, 96), (40, 200)]):
        img = _image(seed, w, h)
        mine = preprocess_image(img, vc)
        ref_pix, ref_grid = _hf_pixels(img, vc)
        assert tuple(ref_grid[0]) == mine.grid
        assert mine.pixels.shape == ref_pix.shape
        assert np.abs(mine.pixels - ref_pix).max() < 1e-5


def test_vision_tower_matches_transformers(tmp_path):
    m, path = _hf_model(tmp_path)
    eng = LLMEngine(EngineConfig(model=path, device="cpu", dtype="float32", max_num_seqs=2,
                                 max_num_batched_tokens=64, num_kv_blocks=64, max_model_len=256), tp=TPGroup())
    vis = eng.runner.model.visual
    vc = _vcfg(eng.model_cfg)
    from hipserve.models.vision import image_geometry

    ims = [preprocess_image(_image(3, 96, 64), vc), preprocess_image(_image(4, 64, 128), vc)]
    pix = np.concatenate([i.pixels for i in ims])
    grids = [i.grid for i in ims]
    emb, ds = vis.forward(torch.from_numpy(pix), image_geometry(grids, vc))
    with torch.no_grad():
        out = m.model.get_image_features(torch.from_numpy(pix), torch.tensor(grids), return_dict=True)
    ref = torch.cat(out.pooler_output)
    assert emb.shape == ref.shape
    torch.testing.assert_close(emb, ref, atol=2e-4, rtol=2e-4)
    assert len(ds) == len(out.deepstack_features) == 2
    for a, b in zip(ds, out.deepstack_features):
        torch.testing.assert_close(a, b, atol=2e-4, rtol=2e-4)


def _prompt(ims, vc):
    ids = [1, 5, 9, VS, IMG, VE, 17, 23, 40, VS, IMG, VE, 11, 12]
    return expand_image_tokens(ids, ims, vc)


def test_mrope_positions_match_transformers(tmp_path):
    m, path = _hf_model(tmp_path)
    mc = ModelConfig.from_hf_dict(m.config.to_dict())
    vc = _vcfg(mc)
    ims = [preprocess_image(_image(5, 96, 64), vc), preprocess_image(_image(6, 64, 160), vc)]
    ids = _prompt(ims, vc)
    st = mm_state(ids, ims, vc)
    tt = torch.tensor([ids])
    pos, delta = m.model.get_rope_index(tt, (tt == IMG).int(), image_grid_thw=torch.tensor([i.grid for i in ims]))
    assert np.array_equal(st.pos3, pos[:, 0].numpy())
    assert st.delta == int(delta)


@pytest.mark.parametrize("chunk", [256, 24])
def test_engine_greedy_with_images_matches_transformers(tmp_path, chunk):
    m, path = _hf_model(tmp_path)
    eng = LLMEngine(EngineConfig(model=path, device="cpu", dtype="float32", max_num_seqs=4,
                                 max_num_batched_tokens=chunk, num_kv_blocks=128, max_model_len=256),
                    tp=TPGroup())
    vc = _vcfg(eng.model_cfg)
    ims = [preprocess_image(_image(8, 96, 64), vc), preprocess_image(_image(9, 64, 96), vc)]
    ids = _prompt(ims, vc)
    text_only = [1, 2, 3, 4, 50, 60, 70]
    sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    res = eng.generate([MultiModalPrompt(ids, ims), text_only], sp)
    pix = torch.from_numpy(np.concatenate([i.pixels for i in ims]))
    grid = torch.tensor([i.grid for i in ims])
    for prompt, (toks, _, reason), mm in ((ids, res[0], True), (text_only, res[1], False)):
        assert reason == "length" and len(toks) == 6
        full = torch.tensor([prompt + list(toks)])
        kw = dict(pixel_values=pix, image_grid_thw=grid, mm_token_type_ids=(full == IMG).int()) if mm else {}
        with torch.no_grad():
            lg = m(full, **kw).logits[0].float()
        for i, t in enumerate(toks):
            row = lg[len(prompt) - 1 + i]
            assert row[t] >= row.max() - 1e-4, (chunk, mm, i, t, int(row.argmax()))


def test_prefix_cache_keys_images_by_content(tmp_path):
    _, path = _hf_model(tmp_path)
    eng = LLMEngine(EngineConfig(model=path, device="cpu", dtype="float32", max_num_seqs=4,
                                 max_num_batched_tokens=256, num_kv_blocks=128, max_model_len=256,
                                 block_size=16), tp=TPGroup())
    vc = _vcfg(eng.model_cfg)
    a = preprocess_image(_image(10, 128, 128), vc)
    b = preprocess_image(_image(11, 128, 128), vc)
    ids = expand_image_tokens([VS, IMG, VE, 5, 6], [a], vc)
    sp = SamplingParams(temperature=0.0, max_tokens=2, ignore_eos=True)
    eng.generate([MultiModalPrompt(ids, [a])], sp)
    s2 = eng.add_request(None, MultiModalPrompt(ids, [b]), sp)
    eng.step()
    assert s2.num_cached_prefix == 0  # same token ids, different image: no KV reuse
    while eng.has_unfinished():
        eng.step()
    s3 = eng.add_request(None, MultiModalPrompt(ids, [a]), sp)
    eng.step()
    assert s3.num_cached_prefix >= 16  # same image: full blocks are reused


def test_chat_image_parts(tmp_path):
    from hipserve.multimodal import load_image
    from hipserve.tokenizer import SyntheticTokenizer, UnsupportedContentError

    buf = io.BytesIO()
    _image(12, 50, 40).save(buf, format="PNG")
    url = "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()
    img = load_image(url)
    assert img.size == (50, 40)
    tk = SyntheticTokenizer(400)
    msgs = [{"role": "user", "content": [{"type": "text", "text": "hi"},
                                         {"type": "image_url", "image_url": {"url": url}}]}]
    with pytest.raises(UnsupportedContentError):
        tk.encode_chat(msgs)
    vc = VisionConfig(image_token_id=IMG, vision_start_token_id=VS, vision_end_token_id=VE)
    ids, urls = tk.encode_chat_mm(msgs, vc)
    assert urls == [url] and ids.count(IMG) == 1 and ids.index(VS) + 1 == ids.index(IMG)


def test_chat_endpoint_with_image(tmp_path):
    """POST /v1/chat/completions with an image_url part on a vision model: 200 and the
    same greedy tokens as the engine-level call; a broken image is a 400, the engine
    stays alive."""
    import asyncio
    import json

    import aiohttp
    from aiohttp import web

    from hipserve.server.api_server import OpenAIServer
    from hipserve.server.async_engine import AsyncEngine

    _, path = _hf_model(tmp_path)
    with open(f"{path}/preprocessor_config.json", "w") as f:
        json.dump({"size": {"shortest_edge": 32 * 32, "longest_edge": 128 * 128}, "patch_size": 16,
                   "image_mean": [0.5] * 3, "image_std": [0.5] * 3}, f)
    buf = io.BytesIO()
    _image(13, 96, 64).save(buf, format="PNG")
    url = "data:image/png;base64," + base64.b64encode(buf.getvalue()).decode()
    msgs = [{"role": "user", "content": [{"type": "image_url", "image_url": {"url": url}},
                                         {"type": "text", "text": "what is this"}]}]

    async def main():
        eng = LLMEngine(EngineConfig(model=path, served_model_name="vl", device="cpu", dtype="float32",
                                     max_num_seqs=4, max_num_batched_tokens=64, num_kv_blocks=128,
                                     max_model_len=256), tp=TPGroup())
        assert eng.model_cfg.vision.min_pixels == 1024
        ae = AsyncEngine(eng)
        ae.start(asyncio.get_running_loop())
        srv = OpenAIServer(ae, "vl", eng.max_model_len)
        runner = web.AppRunner(srv.app())
        await runner.setup()
        site = web.TCPSite(runner, "127.0.0.1", 0)
        await site.start()
        base = f"http://127.0.0.1:{site._server.sockets[0].getsockname()[1]}"
        try:
            async with aiohttp.ClientSession() as s:
                r = await s.post(base + "/v1/chat/completions", json={
                    "model": "vl", "messages": msgs, "max_tokens": 4, "temperature": 0, "ignore_eos": True})
                j = await r.json()
                assert r.status == 200, j
                assert j["usage"]["completion_tokens"] == 4
                assert j["usage"]["prompt_tokens"] > 6  # the image expanded to its merged patches
                bad = [{"role": "user", "content": [{"type": "image_url",
                                                     "image_url": {"url": "data:image/png;base64,AAAA"}}]}]
                r = await s.post(base + "/v1/chat/completions", json={"model": "vl", "messages": bad})
                assert r.status == 400
                assert (await s.get(base + "/health")).status == 200
        finally:
            ae.stop()
            await runner.cleanup()

    asyncio.run(main())


def _tp_worker(rank, world, port, ckpt, q):
    import os

    import torch.distributed as dist

    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from hipserve.config import resolve_model_config
    from hipserve.engine.llm_engine import worker_loop
    from hipserve.engine.model_runner import ModelRunner
    from hipserve.parallel.comm import init_tp

    tp = init_tp(world, backend="gloo", device_type="cpu")
    cfg = _tp_cfg(ckpt, world)
    try:
        if rank == 0:
            eng = LLMEngine(cfg, tp=tp)
            q.put(_tp_generate(eng))
            eng.shutdown()
        else:
            worker_loop(ModelRunner(cfg, resolve_model_config(ckpt), tp), tp)
    finally:
        dist.destroy_process_group()
    q.close()
    q.join_thread()
    os._exit(0)


def _tp_cfg(ckpt, tp):
    return EngineConfig(model=ckpt, device="cpu", dtype="float32", tensor_parallel_size=tp, num_kv_blocks=128,
                        max_model_len=256, max_num_batched_tokens=20, max_num_seqs=4)


def _tp_generate(eng):
    vc = _vcfg(eng.model_cfg)
    ims = [preprocess_image(_image(20, 96, 64), vc), preprocess_image(_image(21, 64, 64), vc)]
    sp = SamplingParams(temperature=0.0, max_tokens=6, ignore_eos=True)
    res = eng.generate([MultiModalPrompt(_prompt(ims, vc), ims), [1, 2, 3, 4, 5]], sp)
    return [r[0] for r in res]


def test_tp2_with_images_matches_tp1(tmp_path):
    """TP=2 over gloo (rank 0 schedules; pixels travel in the step broadcast; every
    rank runs the replicated vision tower; DeepStack features enter the row-parallel
    partial sum on rank 0 only) generates exactly the TP=1 tokens."""
    import socket

    import torch.multiprocessing as mp

    _, ckpt = _hf_model(tmp_path)
    want = _tp_generate(LLMEngine(_tp_cfg(ckpt, 1), tp=TPGroup()))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, ckpt, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want
