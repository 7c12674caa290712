#!/usr/bin/env python3
"""Image-chat throughput of the Qwen3-VL-30B-A3B engine on one MI355X (random-init
weights of the reference's default HF model, its vision tower included): N
concurrent requests, each one synthetic image + a text prompt, greedy-free sampling
of a fixed number of output tokens, engine-level (no HTTP).

    python tools/bench_vl.py --requests 64 --image-size 448 --text-len 256 --output-len 256

Prints one JSON line: wall time, output tok/s, image prefill share, tokens per image.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=64)
    ap.add_argument("--image-size", type=int, default=448)
    ap.add_argument("--text-len", type=int, default=256)
    ap.add_argument("--output-len", type=int, default=256)
    ap.add_argument("--quantization", default=None, choices=[None, "int8", "fp8"])
    a = ap.parse_args()
    import PIL.Image

    from hipserve.config import EngineConfig
    from hipserve.engine.llm_engine import LLMEngine
    from hipserve.engine.request import SamplingParams
    from hipserve.multimodal import MultiModalPrompt, expand_image_tokens, preprocess_image

    extra = {"quantization": a.quantization} if a.quantization else {}
    eng = LLMEngine(EngineConfig(model="qwen3-vl-30b-a3b", load_format="dummy", device="cuda",
                                 max_num_seqs=a.requests, max_num_batched_tokens=8192, max_model_len=4096,
                                 extra=extra))
    vc = eng.model_cfg.vision
    rng = np.random.default_rng(0)
    prompts = []
    for i in range(a.requests):
        img = preprocess_image(PIL.Image.fromarray(
            rng.integers(0, 256, (a.image_size, a.image_size, 3), dtype=np.uint8)), vc)
        text = [int(t) for t in rng.integers(10, 150000, a.text_len)]
        ids = expand_image_tokens([vc.vision_start_token_id, vc.image_token_id, vc.vision_end_token_id] + text,
                                  [img], vc)
        prompts.append(MultiModalPrompt(ids, [img]))
    sp = SamplingParams(temperature=0.8, top_p=0.95, max_tokens=a.output_len, ignore_eos=True)
    eng.generate(prompts[:2], SamplingParams(temperature=0.8, max_tokens=4, ignore_eos=True))  # warm-up
    t0 = time.perf_counter()
    first, n_out = {}, 0
    for p in prompts:
        eng.add_request(None, p, sp)
    while eng.has_unfinished():
        for o in eng.step():
            if o.request_id not in first and o.new_token_ids:
                first[o.request_id] = time.perf_counter() - t0
            n_out += len(o.new_token_ids)
    wall = time.perf_counter() - t0
    ttft = sorted(first.values())
    print(json.dumps({"model": "qwen3-vl-30b-a3b" + (f" {a.quantization.upper()}" if a.quantization else ""),
                      "requests": a.requests, "image": a.image_size, "image_tokens": prompts[0].images[0].num_tokens,
                      "prompt_tokens": len(prompts[0].ids), "output_len": a.output_len,
                      "wall_s": round(wall, 3), "output_tok_per_s": round(n_out / wall, 1),
                      "p50_ttft_ms": round(1e3 * ttft[len(ttft) // 2], 1), "data": "synthetic images, random-init"}),
          flush=True)
    eng.shutdown()


if __name__ == "__main__":
    main()
