"""In-house TP collectives: a thin owner of the HIP-IPC peer
buffers behind ``csrc/kernels/allreduce.hip``.

Every rank allocates one uncached buffer, exports its IPC handle, gathers the
peers' handles over the CPU (gloo) group and maps them; from then on each
collective is a single graph-capturable kernel launch that reads the peers'
staged copies directly over xGMI:

* ``all_reduce(t)``  bf16 sum, one-shot up to ``ONE_SHOT_MAX`` bytes, reduce-
  scatter + all-gather above;
* ``all_gather(t, out)``  [rows, cols] -> [rows, world * cols] (LM-head logits);
* ``add_rmsnorm(...)`` the row-parallel projection epilogue of a decoder layer —
  cross-rank sum of the local (split-K) partials, residual add and RMSNorm in one
  kernel, exchanging fp32 (TP=N within fp32 rounding of TP=1) or bf16.

Each collective has a decode-sized class (64-block grid, lowest latency) and a
prefill-sized class (512-block grid: every CU streams) with their own buffers and
flags. Whether an eager prefill-sized message uses these kernels or RCCL
(all-reduce + local add+RMSNorm) is measured on the node at start-up
(``TPGroup.calibrate_collectives``); messages larger than the registered buffer
always use RCCL, and captured decode graphs always use these kernels. Enabled only after a
self-test against the process-group all-reduce passes on every rank (the
decision is collective), so a node whose IPC / peer mapping misbehaves keeps the
RCCL path instead of producing wrong sums. A barrier timeout anywhere sets a
sticky error that every rank sees (``failed()``, a pinned host word: no device
sync) and the engine turns into a dead pod.
"""
from __future__ import annotations

import logging
import os

import torch
import torch.distributed as dist

log = logging.getLogger("hipserve.custom_ar")

# one-shot -> two-shot crossover (tools/bench_allreduce.py prints the measured one
# for a node) and the default registered message size
ONE_SHOT_MAX = int(os.environ.get("HIPSERVE_CAR_ONE_SHOT_MAX", 256 << 10))
DEFAULT_MAX_BYTES = int(os.environ.get("HIPSERVE_CAR_MAX_BYTES", 8 << 20))


def _device_id(device) -> tuple:
    import socket

    p = torch.cuda.get_device_properties(device)
    uid = getattr(p, "uuid", None)
    return (socket.gethostname(), str(uid) if uid is not None else
            (getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None), device.index))


class CollectiveError(RuntimeError):
    """A custom collective timed out on some rank (a peer died or hung)."""


class CustomAllReduce:
    def __init__(self, rank: int, world: int, cpu_group, device, max_bytes: int = DEFAULT_MAX_BYTES):
        from ..ops import load_library

        load_library()
        self.op = torch.ops.hipserve
        self.rank, self.world, self.device = rank, world, device
        # ranks sharing this GPU (the 1-GPU test box runs a TP group on one device):
        # every block of every sharing rank's collective must be resident at once, so
        # the prefill-sized class gets a smaller grid (<= 1024 blocks per device)
        ids = [None] * world
        dist.all_gather_object(ids, _device_id(device), group=cpu_group)
        self.ranks_per_device = sum(1 for d in ids if d == ids[rank])
        self.nb_large = max(64, min(512, 1024 // self.ranks_per_device))
        with torch.cuda.device(device):
            self.state = int(self.op.car_create(rank, world, max_bytes, self.nb_large))
            self.max_bytes = max_bytes
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

    def supports_gather(self, t: torch.Tensor) -> bool:
        n = t.numel() * t.element_size()
        return (t.is_cuda and t.dim() == 2 and t.is_contiguous() and n <= self.max_bytes
                and (t.shape[1] * t.element_size()) % 2 == 0)

    def all_gather(self, t: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if out is None:
            out = torch.empty(t.shape[0], self.world * t.shape[1], dtype=t.dtype, device=t.device)
        self.op.car_all_gather(self.state, t, out)
        return out

    def norm_fits(self, M: int, N: int, exch_f32: bool) -> bool:
        return bool(self.op.car_norm_fits(self.state, M, N, exch_f32))

    def add_rmsnorm(self, out, residual, x, splits, weight, eps, exch_f32):
        self.op.car_add_rmsnorm(self.state, out, residual, x, splits, weight, eps, exch_f32)

    def failed(self) -> bool:
        return bool(self.op.car_error(self.state))

    def check(self):
        if self.failed():
            raise CollectiveError("a TP collective timed out (a peer rank died or hung); the engine is dead")

    def close(self):
        if self.state:
            self.op.car_destroy(self.state)
            self.state = 0


def self_test(car: CustomAllReduce, group, cpu_group) -> bool:
    """Compare against the process-group all-reduce on a few message sizes (one-shot
    and two-shot) plus the all-gather; collective agreement (all ranks must pass)."""
    ok = True
    try:
        # one-shot, two-shot (small class) and the 512-block large class (> 8 MiB)
        sizes = [8, 4096, 64 * 8192, min(car.max_bytes // 2, 2 << 20)]
        if car.max_bytes >= (12 << 20):
            sizes.append(6 << 20)  # bf16 elements: 12 MiB
        for numel in sizes:
            g = torch.Generator(device=car.device).manual_seed(1234 + 17 * car.rank + numel)
            x = torch.randn(numel, device=car.device, dtype=torch.float32, generator=g).to(torch.bfloat16)
            want = x.float().cpu()
            dist.all_reduce(want, group=cpu_group)
            got = car.all_reduce(x.clone())
            torch.cuda.synchronize(car.device)
            if car.failed() or not torch.allclose(got.float().cpu(), want, atol=0.05, rtol=0.02):
                ok = False
                break
        if ok:
            x = torch.full((3, 64), float(car.rank + 1), device=car.device, dtype=torch.bfloat16)
            got = car.all_gather(x)
            torch.cuda.synchronize(car.device)
            want = torch.cat([torch.full((3, 64), float(r + 1)) for r in range(car.world)], 1)
            ok = not car.failed() and torch.equal(got.float().cpu(), want)
    except Exception as e:  # a broken IPC mapping must not take the engine down
        log.warning("custom all-reduce self-test raised: %s", e)
        ok = False
    flag = [ok] * car.world
    dist.all_gather_object(flag, ok, group=cpu_group)
    return all(flag)
