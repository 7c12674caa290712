"""Tensor-parallel communication (SURVEY §2.D, C1–C4).

One process per GPU (SPMD). ``TPGroup`` wraps a ``torch.distributed`` process
group: backend ``nccl`` on ROCm *is* RCCL, which runs its rings over the xGMI
point-to-point links of an 8xMI355X node; ``gloo`` is used for the CPU tests.

Collectives on the hot path:
  * ``all_reduce``  — sum after the row-parallel o_proj / down_proj (2 per layer)
    and after the vocab-parallel embedding;
  * ``all_gather``  — LM-head logits shards -> full vocab on every rank;
  * ``broadcast_obj`` — step metadata from the rank-0 scheduler to workers, over
    the native shared-memory ring (csrc/runtime/shm_broadcast.cpp) when all ranks
    share a host (always, for TP inside one pod), gloo otherwise / for oversize
    messages.
All ops are in place / into preallocated outputs so decode steps are capturable
into hipGraphs (RCCL collectives are graph-capturable on ROCm).
"""
from __future__ import annotations

import datetime
import os
import pickle
import socket
import uuid

import torch
import torch.distributed as dist


class TPGroup:
    def __init__(self, rank: int = 0, world_size: int = 1, group=None, device=None):
        self.rank = rank
        self.world_size = world_size
        self.group = group
        self.device = device
        self._cpu_group = None
        self._ring = None
        self.custom_ar = None

    SHM_SLOT_BYTES = 8 << 20
    SHM_SLOTS = 4

    def setup_shm_ring(self):
        """Attach the shared-memory step ring (collective over the CPU group)."""
        if self.world_size == 1 or os.environ.get("HIPSERVE_SHM_BROADCAST", "1") == "0":
            return False
        try:
            from .. import runtime
            rt = runtime.native()
        except Exception:  # native runtime unavailable: stay on gloo
            rt = None
        hosts = [None] * self.world_size
        dist.all_gather_object(hosts, (socket.gethostname(), rt is not None), group=self._cpu_group)
        if not all(h == hosts[0][0] and ok for h, ok in hosts):
            return False
        name = [f"/hipserve_tp_{uuid.uuid4().hex[:12]}" if self.rank == 0 else None]
        if self.rank == 0:
            self._ring = rt.ShmBroadcast(name[0], self.world_size - 1, self.SHM_SLOT_BYTES,
                                         self.SHM_SLOTS, 0, True)
        dist.broadcast_object_list(name, src=0, group=self._cpu_group)
        if self.rank != 0:
            self._ring = rt.ShmBroadcast(name[0], self.world_size - 1, self.SHM_SLOT_BYTES,
                                         self.SHM_SLOTS, self.rank, False)
        dist.barrier(group=self._cpu_group)
        return True

    @property
    def is_first(self):
        return self.rank == 0

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over TP ranks: decode-sized bf16 messages through the HIP-IPC
        custom all-reduce (when set up), everything else through RCCL."""
        if self.world_size > 1:
            car = self.custom_ar
            if car is not None and car.supports(t):
                car.all_reduce(t)
            else:
                dist.all_reduce(t, group=self.group)
        return t

    def setup_custom_ar(self, max_bytes: int | None = None) -> bool:
        """Collective: map peer buffers and keep the custom all-reduce only if its
        self-test against RCCL passes on every rank."""
        if self.world_size == 1 or self.device is None or self.device.type != "cuda" \
                or os.environ.get("HIPSERVE_CUSTOM_AR", "1") == "0":
            return False
        from .custom_ar import DEFAULT_MAX_BYTES, CustomAllReduce, self_test
        try:
            car = CustomAllReduce(self.rank, self.world_size, self._cpu_group, self.device,
                                  max_bytes or DEFAULT_MAX_BYTES)
        except Exception as e:
            car = None
            err = str(e)
        else:
            err = ""
        oks = [None] * self.world_size
        dist.all_gather_object(oks, car is not None, group=self._cpu_group)
        if not all(oks):
            if car is not None:
                car.close()
            import logging
            logging.getLogger("hipserve.comm").warning("custom all-reduce unavailable (%s); using RCCL", err)
            return False
        if not self_test(car, self.group, self._cpu_group):
            car.close()
            return False
        self.custom_ar = car
        return True

    def all_gather_lastdim(self, t: torch.Tensor) -> torch.Tensor:
        """[n, V/TP] on every rank -> [n, V] on every rank."""
        if self.world_size == 1:
            return t
        t = t.contiguous()
        if t.device.type == "cpu":  # gloo: list form
            parts = [torch.empty_like(t) for _ in range(self.world_size)]
            dist.all_gather(parts, t, group=self.group)
            return torch.cat(parts, dim=-1)
        parts = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(parts, t, group=self.group)
        return parts.permute(1, 0, 2).reshape(t.shape[0], -1)

    def broadcast_obj(self, obj=None):
        """Rank 0 -> all ranks; returns the object. Shared-memory ring when set up
        (tag byte 0 = inline pickle, 1 = too large, follows over gloo)."""
        if self.world_size == 1:
            return obj
        if self._ring is not None:
            if self.rank == 0:
                data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
                if len(data) + 1 <= self._ring.slot_capacity:
                    self._ring.publish(b"\x00" + data)
                    return obj
                self._ring.publish(b"\x01")
            else:
                msg = self._ring.recv()
                if msg[:1] == b"\x00":
                    return pickle.loads(msg[1:])
        lst = [obj]
        dist.broadcast_object_list(lst, src=0, group=self._cpu_group)
        return lst[0]

    def barrier(self):
        if self.world_size > 1:
            dist.barrier(group=self._cpu_group)


_TP: TPGroup | None = None


def init_tp(world_size: int | None = None, backend: str | None = None, device_type: str = "cuda") -> TPGroup:
    """Initialise the TP group from torchrun-style env vars (RANK/WORLD_SIZE/
    MASTER_ADDR/MASTER_PORT). world_size 1 needs no process group."""
    global _TP
    ws = world_size if world_size is not None else int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if ws == 1:
        dev = torch.device(device_type, int(os.environ.get("LOCAL_RANK", "0"))) if device_type == "cuda" else torch.device("cpu")
        _TP = TPGroup(0, 1, None, dev)
        return _TP
    if backend is None:
        backend = "nccl" if device_type == "cuda" else "gloo"
    if device_type == "cuda":
        local = int(os.environ.get("LOCAL_RANK", rank))
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=ws,
                                timeout=datetime.timedelta(seconds=600))
    g = TPGroup(rank, ws, dist.group.WORLD, dev)
    g._cpu_group = dist.new_group(backend="gloo") if backend != "gloo" else dist.group.WORLD
    g.setup_shm_ring()
    if device_type == "cuda":
        g.setup_custom_ar()
    _TP = g
    return g


def get_tp() -> TPGroup:
    global _TP
    if _TP is None:
        _TP = TPGroup()
    return _TP


def set_tp(g: TPGroup):
    global _TP
    _TP = g
