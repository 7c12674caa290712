"""In-house all-reduce for decode-sized TP messages: a thin owner
of the HIP-IPC peer buffers behind ``csrc/kernels/allreduce.hip``.

Every rank allocates one uncached buffer, exports its IPC handle, gathers the
peers' handles over the CPU (gloo) group and maps them; from then on
``all_reduce(t)`` is a single graph-capturable kernel launch that reads the peers'
staged copies directly over xGMI (one-shot up to ``ONE_SHOT_MAX`` bytes,
reduce-scatter + all-gather above). Messages larger than the registered buffer
(prefill chunks) stay on RCCL, whose ring is bandwidth-optimal there.

Enabled only after a self-test against RCCL passes on every rank (the decision
is collective), so a node whose IPC / peer mapping misbehaves silently keeps the
RCCL path instead of producing wrong sums.
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

log = logging.getLogger("hipserve.custom_ar")

# crossovers (tools/bench_allreduce.py prints the measured ones for a node):
# one-shot -> two-shot, and custom kernel -> RCCL ring (messages above max_bytes)
ONE_SHOT_MAX = int(os.environ.get("HIPSERVE_CAR_ONE_SHOT_MAX", 256 << 10))
DEFAULT_MAX_BYTES = int(os.environ.get("HIPSERVE_CAR_MAX_BYTES", 8 << 20))


class CustomAllReduce:
    def __init__(self, rank: int, world: int, cpu_group, device, max_bytes: int = DEFAULT_MAX_BYTES):
        from ..ops import load_library

        load_library()
        self.op = torch.ops.hipserve
        self.rank, self.world, self.device = rank, world, device
        self.max_bytes = max_bytes
        with torch.cuda.device(device):
            self.state = int(self.op.car_create(rank, world, max_bytes))
            mine = self.op.car_handle(self.state)
        handles = [None] * world
        dist.all_gather_object(handles, bytes(mine.numpy().tobytes()), group=cpu_group)
        with torch.cuda.device(device):
            for p, h in enumerate(handles):
                if p != rank:
                    self.op.car_open(self.state, p, torch.frombuffer(bytearray(h), dtype=torch.uint8))
        dist.barrier(group=cpu_group)

    def supports(self, t: torch.Tensor) -> bool:
        n = t.numel() * t.element_size()
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and n % 16 == 0
                and 0 < n <= self.max_bytes)

    def all_reduce(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum over ranks; in place unless ``out`` is given."""
        out = t if out is None else out
        two_shot = t.numel() * t.element_size() > ONE_SHOT_MAX
        self.op.car_all_reduce(self.state, t, out, two_shot)
        return out

    def failed(self) -> bool:
        return bool(self.op.car_error(self.state))

    def close(self):
        if self.state:
            self.op.car_destroy(self.state)
            self.state = 0


def self_test(car: CustomAllReduce, group, cpu_group) -> bool:
    """Compare against the process-group all-reduce on a few message sizes;
    collective agreement (all ranks must pass)."""
    ok = True
    try:
        for numel in (8, 4096, 64 * 8192, min(car.max_bytes // 2, 2 << 20)):
            g = torch.Generator(device=car.device).manual_seed(1234 + 17 * car.rank + numel)
            x = torch.randn(numel, device=car.device, dtype=torch.float32, generator=g).to(torch.bfloat16)
            want = x.float().clone()
            dist.all_reduce(want, group=group)
            got = car.all_reduce(x.clone())
            torch.cuda.synchronize(car.device)
            if car.failed() or not torch.allclose(got.float(), want, atol=0.05, rtol=0.02):
                ok = False
                break
    except Exception as e:  # a broken IPC mapping must not take the engine down
        log.warning("custom all-reduce self-test raised: %s", e)
        ok = False
    flag = [ok] * car.world
    dist.all_gather_object(flag, ok, group=cpu_group)
    return all(flag)
