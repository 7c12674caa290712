"""Probe torch._grouped_mm on the GPU for the MoE prefill expert GEMMs
(Qwen3-30B-A3B shapes: 128 experts, H 2048, expert width 768; Mixtral: 8 experts,
H 4096, width 14336): correctness vs a per-expert loop and time of both.

    python tools/bench_grouped_mm.py
"""
import json
import time

import torch


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


def main():
    dev = torch.device("cuda", 0)
    for name, E, H, I, P in [("qwen3-moe", 128, 2048, 768, 65536), ("mixtral", 8, 4096, 14336, 16384)]:
        torch.manual_seed(0)
        w13 = torch.randn(E, 2 * I, H, device=dev, dtype=torch.bfloat16) * 0.02
        ids = torch.randint(0, E, (P,), device=dev)
        counts = torch.bincount(ids, minlength=E)
        offs = torch.cumsum(counts, 0).to(torch.int32)
        xs = torch.randn(P, H, device=dev, dtype=torch.bfloat16)
        b = w13.transpose(1, 2)
        row = {"model": name, "E": E, "P": P}
        try:
            y = torch._grouped_mm(xs, b, offs=offs)
            cl = counts.tolist()
            ref, a = [], 0
            for e in range(E):
                ref.append(xs[a:a + cl[e]] @ w13[e].T)
                a += cl[e]
            ref = torch.cat(ref)
            row["max_rel_err"] = float((y.float() - ref.float()).abs().max() / ref.float().abs().max())
            row["grouped_us"] = round(timeit(lambda: torch._grouped_mm(xs, b, offs=offs)), 1)
        except Exception as e:  # noqa: BLE001
            row["grouped_error"] = str(e)[:300]

        def loop():
            a = 0
            for e, c in enumerate(cl):
                if c:
                    torch.nn.functional.linear(xs[a:a + c], w13[e])
                a += c

        cl = counts.tolist()
        row["loop_us"] = round(timeit(loop), 1)
        flops = 2 * P * H * 2 * I
        for k in ("grouped_us", "loop_us"):
            if k in row:
                row[k.replace("_us", "_TFLOPs")] = round(flops / row[k] / 1e6, 1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
