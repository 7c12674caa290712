"""Native shared-memory step ring (csrc/runtime/shm_broadcast.cpp) and the TP
step broadcast built on it, multi-process on CPU."""
import multiprocessing as mp
import os
import socket
import uuid

import pytest

from hipserve import runtime


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _reader(name, rank, readers, n, q):
    rt = runtime.native()
    ring = rt.ShmBroadcast(name, readers, 4096, 3, rank, False)
    got = [ring.recv(30.0) for _ in range(n)]
    q.put((rank, [g if g is None else bytes(g) for g in got]))


def test_ring_ordering_and_backpressure():
    rt = runtime.native()
    name = f"/hipserve_test_{uuid.uuid4().hex[:8]}"
    readers, n = 3, 200
    w = rt.ShmBroadcast(name, readers, 4096, 3, 0, True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_reader, args=(name, r, readers, n, q)) for r in range(1, readers + 1)]
    for p in ps:
        p.start()
    msgs = [os.urandom(1 + (i * 37) % 4000) for i in range(n)]
    for m in msgs:  # 3 slots << 200 messages: publish must wait for slow readers
        w.publish(m)
    res = dict(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(30)
    assert all(res[r] == msgs for r in range(1, readers + 1))
    with pytest.raises(Exception):
        w.publish(b"x" * 5000)  # larger than a slot


def _tp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from hipserve.parallel.comm import TPGroup, init_tp
    TPGroup.SHM_SLOT_BYTES = 1 << 14
    tp = init_tp(world, backend="gloo", device_type="cpu")
    out = []
    for i in range(50):
        obj = {"i": i, "blob": b"z" * (100 if i % 10 else 40000)} if rank == 0 else None
        got = tp.broadcast_obj(obj)
        out.append((got["i"], len(got["blob"])))
    q.put((rank, tp._ring is not None, out))
    import torch.distributed as dist
    dist.barrier()
    dist.destroy_process_group()


def test_tp_broadcast_over_ring_with_gloo_fallback():
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_tp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in ps:
        r, ring, out = q.get(timeout=120)
        res[r] = (ring, out)
    for p in ps:
        p.join(60)
    want = [(i, 100 if i % 10 else 40000) for i in range(50)]
    for r in range(world):
        assert res[r][0], "shared-memory ring not set up"
        assert res[r][1] == want
