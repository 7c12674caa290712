#!/usr/bin/env python3
"""All-reduce µbench for the TP thresholds (SURVEY §2.D "Distributed communication
backend", §7.2 step 7): RCCL ring vs the in-house HIP-IPC one-shot / two-shot
kernels (csrc/kernels/allreduce.hip) over a sweep of bf16 message sizes.

One process per GPU, launched like the engine:

    torchrun --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py

Rank 0 prints a markdown table (µs per call, max over ranks, and the algorithmic
bus bandwidth 2(N-1)/N * bytes / t) and the one-shot -> two-shot crossover
(``HIPSERVE_CAR_ONE_SHOT_MAX``). ``--norm H`` adds the row-parallel epilogue sweep:
the fused cross-rank add+RMSNorm kernel (``car_norm``: 64-block class up to 512
rows, 512-block class above) against RCCL all-reduce + local fused add+RMSNorm
at [M, H] bf16 — the comparison the engine's start-up calibration makes
(``TPGroup.calibrate_collectives``). With fewer GPUs than ranks (``--shared-gpu``:
every rank on cuda:0, the 1-GPU rehearsal) RCCL is skipped — it refuses two ranks
on one device — and the custom kernels run over intra-device IPC.

Graph mode: every rank captures and instantiates its graph, then the ranks meet at
a barrier before the timed replays. (Round 1's table timed from a barrier placed
BEFORE the capture, so the first size's replay also waited out the other rank's
capture skew: the 57 us entry at 16 KiB in ``profiles/r1_allreduce_shared_gpu.md``.)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SIZES = [16 << 10, 64 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 32 << 20, 128 << 20]
NORM_ROWS = [1, 16, 64, 256, 512, 1024, 2048, 4096, 8192]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--max-custom-bytes", type=int, default=128 << 20)
    ap.add_argument("--norm", type=int, default=0, help="hidden size of the add+RMSNorm sweep (0: skip)")
    ap.add_argument("--shared-gpu", action="store_true", help="all ranks on cuda:0 (no RCCL)")
    ap.add_argument("--graph", action="store_true", help="time hipGraph replays of --iters calls")
    ap.add_argument("--out", default=None, help="also write one JSON line per (size, mode)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from hipserve.parallel.custom_ar import CustomAllReduce

    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dev = torch.device("cuda", 0 if args.shared_gpu else local)
    torch.cuda.set_device(dev)
    use_rccl = not args.shared_gpu
    dist.init_process_group("nccl" if use_rccl else "gloo", rank=rank, world_size=world)
    cpu = dist.new_group(backend="gloo")
    car = CustomAllReduce(rank, world, cpu, dev, max_bytes=args.max_custom_bytes) if world > 1 else None

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        dist.barrier(group=cpu)
        if args.graph:
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                fn()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                for _ in range(args.iters):
                    fn()
            torch.cuda.synchronize()
            dist.barrier(group=cpu)  # every rank's graph is instantiated: no capture skew in the timing
            run = g.replay
        else:
            def run():
                for _ in range(args.iters):
                    fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        run()
        b.record()
        b.synchronize()
        us = torch.tensor([a.elapsed_time(b) * 1000.0 / args.iters])
        dist.all_reduce(us, op=dist.ReduceOp.MAX, group=cpu)
        return float(us)

    rows = []
    for nbytes in SIZES:
        x = torch.randn(nbytes // 2, device=dev).to(torch.bfloat16)
        out = torch.empty_like(x)
        res = {}
        if use_rccl:
            res["rccl"] = timed(lambda: dist.all_reduce(x))
        if car is not None and car.supports(x):
            if nbytes <= max(args.max_custom_bytes, 1):
                res["one_shot"] = timed(lambda: car.op.car_all_reduce(car.state, x, out, False))
                res["two_shot"] = timed(lambda: car.op.car_all_reduce(car.state, x, out, True))
        rows.append((nbytes, res))
        if rank == 0 and args.out:
            with open(args.out, "a") as f:
                for mode, us in res.items():
                    f.write(json.dumps({"bytes": nbytes, "mode": mode, "us": round(us, 2), "world": world,
                                        "graph": args.graph, "shared_gpu": args.shared_gpu}) + "\n")
    norm_rows = []
    if args.norm and car is not None:
        from hipserve.ops import get_ops

        ops = get_ops(dev)
        H = args.norm
        w = torch.ones(H, device=dev, dtype=torch.bfloat16)
        for M in NORM_ROWS:
            if not car.norm_fits(M, H, M <= 512):
                continue
            exch = M <= 512  # the engine's default: fp32 exchange for decode batches
            x = (torch.randn(M, H, device=dev) * 0.1).to(torch.bfloat16)
            resid = torch.zeros(M, H, device=dev, dtype=torch.bfloat16)
            o = torch.empty_like(resid)
            res = {"car_norm": timed(lambda: car.add_rmsnorm(o, resid, x, 1, w, 1e-5, exch))}
            if use_rccl:
                def rc():
                    h = x.clone()
                    dist.all_reduce(h)
                    ops.fused_add_rmsnorm(o, h, resid, w, 1e-5)
                res["rccl+norm"] = timed(rc)
            norm_rows.append((M, res))
            if rank == 0 and args.out:
                with open(args.out, "a") as f:
                    for mode, us in res.items():
                        f.write(json.dumps({"rows": M, "hidden": H, "mode": mode, "us": round(us, 2), "world": world,
                                            "graph": args.graph, "shared_gpu": args.shared_gpu}) + "\n")
    if car is not None:
        car.close()

    if rank == 0:
        modes = ["rccl", "one_shot", "two_shot"]
        bw = 2 * (world - 1) / max(world, 1)
        print(f"# all-reduce sweep: world {world}, bf16, {'hipGraph' if args.graph else 'eager'}, "
              f"{args.iters} calls/size{' (shared GPU)' if args.shared_gpu else ''}\n")
        print("| bytes | " + " | ".join(f"{m} us (GB/s)" for m in modes) + " |")
        print("|---:|" + "---:|" * len(modes))
        for nbytes, res in rows:
            cells = []
            for m in modes:
                if m in res:
                    cells.append(f"{res[m]:.1f} ({bw * nbytes / res[m] / 1e3:.0f})")
                else:
                    cells.append("—")
            print(f"| {nbytes} | " + " | ".join(cells) + " |")
        one_max = max((n for n, r in rows if "one_shot" in r and r["one_shot"] <= r.get("two_shot", 1e30)),
                      default=None)
        car_max = max((n for n, r in rows if "rccl" in r
                       and min(r.get("one_shot", 1e30), r.get("two_shot", 1e30)) < r["rccl"]), default=None)
        print(f"\nsuggested HIPSERVE_CAR_ONE_SHOT_MAX={one_max}")
        if use_rccl:
            print(f"in-house all-reduce faster than RCCL up to {car_max} bytes")
        if norm_rows:
            print(f"\n# add+RMSNorm epilogue [M, {args.norm}] bf16 (fp32 exchange up to 512 rows)\n")
            print("| rows | MiB | car_norm us (GB/s) | rccl all-reduce + norm us |")
            print("|---:|---:|---:|---:|")
            for M, res in norm_rows:
                nb = M * args.norm * 2
                c = res["car_norm"]
                r = f"{res['rccl+norm']:.1f}" if "rccl+norm" in res else "—"
                print(f"| {M} | {nb / 2**20:.2f} | {c:.1f} ({bw * nb / c / 1e3:.0f}) | {r} |")
    dist.barrier(group=cpu)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
