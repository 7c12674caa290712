"""In-house TP collectives (csrc/kernels/allreduce.hip) with 2 or 4 ranks sharing
the one GPU of the test box (HIP IPC within a device; handles exchanged over
gloo): one-shot and two-shot all-reduce vs the exact per-rank inputs, the logits
all-gather, the fused cross-rank add+RMSNorm epilogue vs an fp32 torch reference
(fp32 / bf16 exchange, split-K partial / bf16 inputs, bf16 / fp32 norm weights),
interleaved message sizes (the per-block paired barriers must hold when the
element partition changes between calls), hipGraph capture, and the sticky error
of a timed-out barrier. A real 8xMI355X node exercises the xGMI path."""
import multiprocessing as mp
import os
import socket

import pytest

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(numel, rank, it, torch):
    g = torch.Generator().manual_seed(1000 * it + 10 * rank + numel % 97)
    return (torch.randint(-8, 9, (numel,), generator=g).float() / 4).to(torch.bfloat16)


def _norm_inputs(rank, S, M, N, it, torch):
    g = torch.Generator().manual_seed(7 + 31 * rank + 131 * it + M)
    x = torch.randn(S, M, N, generator=g) * 0.5
    g2 = torch.Generator().manual_seed(99 + it + M)  # identical on every rank
    res = (torch.randn(M, N, generator=g2)).to(torch.bfloat16)
    w = (1.0 + 0.1 * torch.randn(N, generator=g2))
    return x, res, w


def _norm_ref(xs, res, w, eps, exch_f32, torch):
    """fp32 reference of the fused epilogue with the kernel's rounding points."""
    locs = [x.sum(0) for x in xs]
    if not exch_f32:
        locs = [v.to(torch.bfloat16).float() for v in locs]
    h = sum(locs).to(torch.bfloat16).float()
    r = (h + res.float()).to(torch.bfloat16)
    rf = r.float()
    out = (rf * torch.rsqrt(rf.pow(2).mean(-1, keepdim=True) + eps) * w.float()).to(torch.bfloat16)
    return out, r


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      HIPSERVE_CAR_TIMEOUT_S="3")
    import torch
    import torch.distributed as dist
    from hipserve.parallel.custom_ar import CustomAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    res = {}
    try:
        car = CustomAllReduce(rank, world, dist.group.WORLD, dev, max_bytes=24 << 20)
        # all-reduce, one-shot and two-shot, sizes interleaved with the other kinds;
        # 5M / 9M elements (10 / 18 MiB) run on the 512-block prefill-sized class
        for numel in (8, 1000 * 8, 64 * 4096, 5 << 20, 1 << 20, 24, 9 << 20, 3 * 4096):
            for it in range(3):
                x = _inputs(numel, rank, it, torch).to(dev)
                want = sum(_inputs(numel, r, it, torch).float() for r in range(world))
                car.all_reduce(x)  # in place
                torch.cuda.synchronize()
                res[("ar", numel, it)] = bool(torch.equal(x.float().cpu(), want))
        # all-gather (logits shards): 16-B rows, 4-B rows and 2-B rows
        for rows, cols, dt in ((5, 4008, torch.bfloat16), (16, 16032, torch.float32), (3, 6, torch.bfloat16),
                               (2, 7, torch.bfloat16)):
            x = (torch.arange(rows * cols, dtype=torch.float32).view(rows, cols) + 100000 * rank).to(dt)
            got = car.all_gather(x.to(dev))
            torch.cuda.synchronize()
            want = torch.cat([(torch.arange(rows * cols, dtype=torch.float32).view(rows, cols) + 100000 * r).to(dt)
                              for r in range(world)], 1)
            res[("ag", rows, cols, str(dt))] = bool(torch.equal(got.cpu(), want))
        # fused cross-rank add + RMSNorm
        eps = 1e-5
        # rows > 512: the 512-block class (2 or more rows per block, 64..256 threads a row)
        for S, M, N, exch, wf32, bf_in in ((4, 64, 2048, True, False, False), (1, 1, 1024, True, False, False),
                                           (1, 1024, 4096, False, False, True), (2, 70, 1024, False, True, False),
                                           (1, 130, 4096, True, True, True), (1, 700, 512, False, False, True),
                                           (1, 16, 512, False, False, True), (1, 1500, 2048, False, True, True)):
            for it in range(2):
                xs = [_norm_inputs(r, S, M, N, it, torch)[0] for r in range(world)]
                _, resid, w = _norm_inputs(rank, S, M, N, it, torch)
                xin = xs[rank].to(torch.bfloat16) if bf_in else xs[rank]
                ref_xs = [x.to(torch.bfloat16).float() for x in xs] if bf_in else xs
                want_out, want_res = _norm_ref(ref_xs, resid, w, eps, exch, torch)
                wt = w.to(dev) if wf32 else w.to(torch.bfloat16).to(dev)
                if not wf32:
                    want_out, want_res = _norm_ref(ref_xs, resid, w.to(torch.bfloat16).float(), eps, exch, torch)
                r_d = resid.to(dev)
                out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
                car.add_rmsnorm(out, r_d, xin.to(dev).contiguous(), S, wt, eps, exch)
                torch.cuda.synchronize()
                d_out = (out.float().cpu() - want_out.float()).abs().max().item()
                d_res = (r_d.float().cpu() - want_res.float()).abs().max().item()
                res[("norm", S, M, N, exch, wf32, bf_in, it)] = bool(d_out <= 0.0625 and d_res <= 0.0625)
        # hipGraph capture: the call counters live on the device
        numel = 64 * 4096
        x = torch.zeros(numel, device=dev, dtype=torch.bfloat16)
        out = torch.empty_like(x)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            car.all_reduce(x, out)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            car.all_reduce(x, out)
            car.all_reduce(x[:64], out[:64])
        for it in range(4):
            x.copy_(_inputs(numel, rank, 10 + it, torch).to(dev))
            g.replay()
            torch.cuda.synchronize()
            want = sum(_inputs(numel, r, 10 + it, torch).float() for r in range(world))
            res[("graph", it)] = bool(torch.equal(out.float().cpu(), want))
        res["error_flag_clean"] = not car.failed()
        # sticky error: rank 0 calls alone -> times out; afterwards every rank fails fast
        dist.barrier()
        if rank == 0:
            car.all_reduce(torch.ones(64, device=dev, dtype=torch.bfloat16))
            torch.cuda.synchronize()
        dist.barrier()
        if rank != 0:
            car.all_reduce(torch.ones(64, device=dev, dtype=torch.bfloat16))
            torch.cuda.synchronize()
        res["error_flag_raised"] = car.failed()
        car.close()
    except Exception as e:  # report instead of hanging the parent
        import traceback
        res["exception"] = traceback.format_exc()
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_custom_collectives_shared_gpu(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=110) for _ in ps)
    for p in ps:
        p.join(30)
    for r in range(world):
        res = out[r]
        assert "exception" not in res, res["exception"]
        assert res.pop("error_flag_clean"), "a barrier timed out"
        assert res.pop("error_flag_raised"), "the missing-peer timeout did not set the sticky error"
        assert all(res.values()), {k: v for k, v in res.items() if not v}
