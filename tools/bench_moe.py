"""Time one Mixtral-8x7B MoE layer (router -> experts -> combine) at decode batch
sizes on the three expert-GEMM paths of LlamaModel.moe_hip: the legacy 16-row
gathered GEMM, the expert decode GEMM on row-major weights, and on packed weights
(GLU epilogue + split-K partials). Graph-timed; effective TB/s counts the expert
weight bytes of the experts that received tokens.

    python tools/bench_moe.py [--tokens 1,8,32,64] [--check]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_ops import graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="1,8,32,64")
    ap.add_argument("--layers", type=int, default=2, help="distinct layers cycled (defeats the MALL)")
    ap.add_argument("--check", action="store_true", help="compare each path with the torch MoE")
    a = ap.parse_args()

    from hipserve import ops as ops_mod
    from hipserve.config import PRESETS
    from hipserve.models.llama import LayerWeights, LlamaModel
    from hipserve.parallel.comm import TPGroup

    dev = torch.device("cuda:0")
    ops = ops_mod.get_ops(dev)
    cfg = PRESETS["mixtral-8x7b"]
    E, H, I, k = cfg.num_experts, cfg.hidden_size, cfg.intermediate_size, cfg.num_experts_per_tok
    m = LlamaModel(cfg, TPGroup(0, 1, None, dev), dev, torch.bfloat16, ops)
    torch.manual_seed(0)
    lws = []
    for _ in range(a.layers):
        lw = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None,
                          router=torch.randn(E, H, device=dev, dtype=torch.bfloat16) * 0.05,
                          w13=(torch.rand(E, 2 * I, H, device=dev, dtype=torch.bfloat16) - 0.5) * 0.04,
                          w2=(torch.rand(E, H, I, device=dev, dtype=torch.bfloat16) - 0.5) * 0.02)
        lws.append(lw)
    m.layers = lws
    packed_bytes = m.pack_moe_weights()
    print(f"packed {packed_bytes / 2**30:.1f} GiB", flush=True)
    packs = [lw.moe_packed for lw in lws]
    expert_bytes = 3 * H * I * 2
    orig_ok = LlamaModel._moe_decode_ok

    for T in [int(t) for t in a.tokens.split(",")]:
        x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
        with torch.no_grad():
            ids = torch.topk(torch.nn.functional.linear(x, lws[0].router).float(), k, dim=-1).indices
        active = int(torch.unique(ids).numel())
        row = {"T": T, "active_experts": active}
        for mode in ("legacy", "rowmajor", "packed"):
            for lw, p in zip(lws, packs):
                lw.moe_packed = p if mode == "packed" else None
            LlamaModel._moe_decode_ok = (lambda self, lw: False) if mode == "legacy" else orig_ok

            def fn():
                for lw in lws:
                    m.moe_hip(x, lw)

            us = graph_time(fn, n=10) / len(lws)
            row[f"{mode}_us"] = round(us, 1)
            row[f"{mode}_TBps"] = round(active * expert_bytes / us / 1e6, 2)
            if a.check:
                got = m.moe_hip(x, lws[0]).float()
                m.ops = type("R", (), {"name": "reference", "silu_and_mul": ops.silu_and_mul})()
                want = m.moe(x, lws[0]).float()
                m.ops = ops
                row[f"{mode}_maxerr"] = round((got - want).abs().max().item() / want.abs().max().item(), 4)
        LlamaModel._moe_decode_ok = orig_ok
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
