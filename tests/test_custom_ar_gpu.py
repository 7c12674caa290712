"""Custom all-reduce (csrc/kernels/allreduce.hip) with 2 ranks sharing the one
GPU of the test box (HIP IPC within a device; handles exchanged over gloo):
one-shot and two-shot sums vs the exact per-rank inputs, in place, under a
hipGraph with changing inputs. A real 8xMI355X node exercises the xGMI path."""
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


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    from hipserve.parallel.custom_ar import CustomAllReduce

    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    res = {}
    try:
        car = CustomAllReduce(rank, world, dist.group.WORLD, dev, max_bytes=4 << 20)
        for numel in (8, 1000 * 8, 64 * 4096, 1 << 20):  # 16 B .. 2 MiB (one-shot and two-shot)
            for it in range(3):
                x = _inputs(numel, rank, it, torch).to(dev)
                want = sum(_inputs(numel, r, it, torch).float() for r in range(world))
                car.all_reduce(x)  # in place
                torch.cuda.synchronize()
                res[(numel, it)] = bool(torch.equal(x.float().cpu(), want))
        # hipGraph capture: the call counter lives on the device
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
        for it in range(4):
            x.copy_(_inputs(numel, rank, 10 + it, torch).to(dev))
            g.replay()
            torch.cuda.synchronize()
            want = sum(_inputs(numel, r, 10 + it, torch).float() for r in range(world))
            res[("graph", it)] = bool(torch.equal(out.float().cpu(), want))
        res["error_flag"] = car.failed()
        car.close()
    except Exception as e:  # report instead of hanging the parent
        res["exception"] = repr(e)
    q.put((rank, res))
    dist.barrier()
    dist.destroy_process_group()


def test_custom_all_reduce_two_ranks_one_gpu():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(60)
    for r in range(world):
        res = out[r]
        assert "exception" not in res, res
        assert not res.pop("error_flag"), "a barrier timed out"
        assert all(res.values()), {k: v for k, v in res.items() if not v}
