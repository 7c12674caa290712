#!/usr/bin/env python3
"""Qwen3-VL vision tower throughput on one MI355X (random-init weights of the
Qwen3-VL-30B-A3B / 235B tower: depth 27, hidden 1152, 16 heads of 72, MLP 4304,
DeepStack after blocks 8/16/24, output 2048): bf16 forward of a batch of synthetic
images, graph-free eager (one launch per op, like the engine's prefill).

    python tools/bench_vision.py --size 1024 --images 4 --iters 10

Prints one JSON line: ms per batch, images/s, patches/s and the achieved dense
TFLOP/s (GEMMs + attention, counted from the shapes).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def flops(cfg, grids) -> float:
    C, I, nh = cfg.hidden_size, cfg.intermediate_size, cfg.num_heads
    Np = sum(t * h * w for t, h, w in grids)
    gemm = 2 * Np * (cfg.patch_dim * C + cfg.depth * (3 * C * C + C * C + 2 * C * I))
    attn = cfg.depth * sum(t * 4 * (h * w) ** 2 * C for t, h, w in grids)
    M = C * cfg.spatial_merge_size ** 2
    merge = (1 + len(cfg.deepstack_visual_indexes)) * 2 * (Np // 4) * (M * M + M * cfg.out_hidden_size)
    return float(gemm + attn + merge)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024, help="square image side in pixels")
    ap.add_argument("--images", type=int, default=4)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    import torch

    from hipserve.config import VisionConfig
    from hipserve.models.vision import VisionTower, image_geometry
    from hipserve.multimodal import preprocess_image
    from hipserve.ops import get_ops

    import PIL.Image

    dev = torch.device("cuda", 0)
    cfg = VisionConfig()
    vt = VisionTower(cfg, dev, torch.bfloat16, get_ops(dev))
    vt.allocate_random(0)
    rng = np.random.default_rng(0)
    ims = [preprocess_image(PIL.Image.fromarray(rng.integers(0, 256, (a.size, a.size, 3), dtype=np.uint8)), cfg)
           for _ in range(a.images)]
    pix = torch.from_numpy(np.concatenate([i.pixels for i in ims])).to(dev)
    geo = image_geometry([i.grid for i in ims], cfg)
    for _ in range(a.warmup):
        vt.forward(pix, geo)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        emb, ds = vt.forward(pix, geo)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    f = flops(cfg, [i.grid for i in ims])
    print(json.dumps({"images": a.images, "size": a.size, "patches_per_image": int(ims[0].pixels.shape[0]),
                      "tokens_per_image": ims[0].num_tokens, "ms_per_batch": round(dt * 1e3, 3),
                      "images_per_s": round(a.images / dt, 2), "patches_per_s": round(pix.shape[0] / dt),
                      "tflops": round(f / dt / 1e12, 1), "out": list(emb.shape), "deepstack": len(ds)}),
          flush=True)


if __name__ == "__main__":
    main()
