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


def rccl_crossover(results) -> int | None:
    """Pure decision of ``TPGroup.calibrate_collectives``: ``results`` are (rows,
    in-house kernel time, RCCL time) by increasing rows (max over ranks). Returns the
    smallest row count from which RCCL is faster at EVERY larger measured size, None
    when the in-house kernel wins at the largest size (a size where RCCL wins but a
    larger one where it loses does not move the crossover down: the routing is a
    single threshold)."""
    res = sorted(results)
    for i, (M, _, _) in enumerate(res):
        if all(tr < tc for _, tc, tr in res[i:]):
            return M
    return None


def route_rccl(rows: int, min_rows: int | None, floor_rows: int, backend: str | None, capturing: bool) -> bool:
    """Pure routing of one eager message of ``rows`` rows: RCCL only on an RCCL group,
    outside a hipGraph capture, at or above the calibrated crossover AND above
    ``floor_rows`` (the largest decode-graph batch): every decode-sized message stays
    on the in-house kernel whether its step runs captured or eager (penalty
    initialisation steps run eager), so graph and eager decode steps reduce in the
    same order."""
    return (min_rows is not None and backend == "nccl" and not capturing
            and rows >= min_rows and rows > floor_rows)


class TPGroup:
    def __init__(self, rank: int = 0, world_size: int = 1, group=None, device=None):
        self.rank = rank
        self.world_size = world_size
        self.group = group
        self.device = device
        self._cpu_group = None
        self._ring = None
        self.custom_ar = None
        self.backend = dist.get_backend(group) if group is not None else None
        # row-parallel epilogues exchange fp32 partial sums up to this many rows (all
        # decode batches), bf16 above (prefill chunks: half the xGMI bytes);
        # exact_reduce forces fp32 everywhere (prefill GEMMs then write fp32 too)
        self.fp32_exchange_rows = int(os.environ.get("HIPSERVE_TP_FP32_ROWS", 512))
        self.exact_reduce = os.environ.get("HIPSERVE_TP_EXACT", "0") == "1"
        # eager (prefill-sized) messages of at least this many rows go through RCCL
        # instead of the in-house kernels; set per node by calibrate_collectives()
        # (None: always in-house). HIPSERVE_CAR_RCCL_MIN_ROWS overrides (-1: never).
        self.rccl_min_rows: int | None = None
        # messages of at most this many rows always take the in-house kernels (set by
        # the runner to its largest decode-graph batch)
        self.rccl_floor_rows = self.fp32_exchange_rows
        self.collective_report: list[dict] = []

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

    def _uncapturable(self, what: str):
        """A process-group collective inside a hipGraph capture is only legal on
        RCCL; with a gloo device group (the shared-GPU TP tests) every captured
        collective must be an in-house kernel."""
        if self.backend == "gloo" and torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"{what} is not covered by the custom collectives and cannot be "
                               "captured on a gloo process group (register a larger custom buffer)")

    def _use_rccl(self, rows: int) -> bool:
        """Route an eager message of ``rows`` rows through RCCL (calibrated crossover;
        captured decode graphs always use the in-house kernels)."""
        capturing = torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()
        return route_rccl(rows, self.rccl_min_rows, self.rccl_floor_rows, self.backend, capturing)

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over TP ranks: bf16 messages that fit the registered buffer
        through the HIP-IPC custom all-reduce (when set up) below the calibrated
        RCCL crossover, everything else through the process group (RCCL)."""
        if self.world_size > 1:
            car = self.custom_ar
            if car is not None and car.supports(t) and not self._use_rccl(t.shape[0] if t.dim() > 1 else 1):
                car.all_reduce(t)
            else:
                self._uncapturable("all_reduce")
                dist.all_reduce(t, group=self.group)
        return t

    def add_rmsnorm(self, out, residual, x, splits, weight, eps, ops=None, exch_f32: bool | None = None):
        """Row-parallel projection epilogue (o_proj / down_proj / MoE combine):
        h = sum over ranks of this rank's partial output ``x`` (fp32 split-K partials
        [S, M, N] or bf16 [M, N]), residual += bf16(h), out = RMSNorm(residual).
        One in-house kernel when the custom collectives are up; otherwise a local
        reduce + all-reduce + fused_add_rmsnorm (same rounding points)."""
        M, N = residual.shape
        car = self.custom_ar
        if exch_f32 is None:
            exch_f32 = self.exact_reduce or M <= self.fp32_exchange_rows
        if car is not None and x.is_cuda and not self._use_rccl(M):
            if not car.norm_fits(M, N, exch_f32) and exch_f32 and not self.exact_reduce:
                exch_f32 = False
            if car.norm_fits(M, N, exch_f32):
                car.add_rmsnorm(out, residual, x, splits, weight, eps, exch_f32)
                return out
        if x.dtype == torch.float32 and x.numel() == splits * M * N and residual.dtype != torch.float32:
            h = x.view(splits, M, N).sum(0)
            if not (exch_f32 and self.world_size > 1):
                h = h.to(residual.dtype)
        else:
            h = x.view(M, N)
        if self.world_size > 1:
            self._uncapturable("add_rmsnorm")
            dist.all_reduce(h, group=self.group)
        (ops or _default_ops(residual.device)).fused_add_rmsnorm(out, h.to(residual.dtype), residual, weight, eps)
        return out

    def check(self):
        """Raise if a custom collective timed out on any rank (sticky, host-visible)."""
        if self.custom_ar is not None:
            self.custom_ar.check()

    def ensure_custom_ar(self, max_bytes: int) -> bool:
        """Collective (every rank, same argument): (re)create the custom collectives
        with at least ``max_bytes`` per message."""
        car = self.custom_ar
        if car is not None and car.max_bytes >= max_bytes:
            return True
        if car is not None:
            self.barrier()
            car.close()
            self.custom_ar = None
        return self.setup_custom_ar(max_bytes)

    def setup_custom_ar(self, max_bytes: int | None = None) -> bool:
        """Collective: map peer buffers and keep the custom all-reduce only if its
        self-test against the process group passes on every rank."""
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

    def calibrate_collectives(self, N: int, max_rows: int, dtype=torch.bfloat16) -> list[dict]:
        """Collective, at start-up on a TP>1 RCCL node with the in-house kernels up:
        time the fused cross-rank add+RMSNorm of an eager [M, N] bf16 message both
        ways — the in-house IPC kernel vs RCCL all-reduce + local fused add+RMSNorm —
        at prefill-sized row counts, and route M >= the smallest row count from which
        RCCL is faster at every larger measured size through RCCL. Timings are the max
        over ranks, so every rank takes the same decision."""
        env = os.environ.get("HIPSERVE_CAR_RCCL_MIN_ROWS")
        if env is not None:
            v = int(env)
            self.rccl_min_rows = None if v < 0 else v
            return []
        car = self.custom_ar
        if self.world_size == 1 or car is None or self.backend != "nccl":
            return []
        dev = self.device
        ops = _default_ops(dev)
        rows = [m for m in (256, 512, 1024, 2048, 4096, 8192, 16384) if m <= max_rows] or [max_rows]
        w = torch.ones(N, dtype=dtype, device=dev)
        res: list[tuple[int, float, float]] = []
        self.rccl_min_rows = None
        for M in rows:
            if not car.norm_fits(M, N, False):
                break
            g = torch.Generator(device=dev).manual_seed(M + self.rank)
            x = (torch.randn(M, N, device=dev, generator=g) * 0.1).to(dtype)
            resid = torch.zeros(M, N, dtype=dtype, device=dev)
            out = torch.empty_like(resid)

            def run_car():
                car.add_rmsnorm(out, resid, x, 1, w, 1e-5, False)

            def run_rccl():
                h = x.clone()
                dist.all_reduce(h, group=self.group)
                ops.fused_add_rmsnorm(out, h, resid, w, 1e-5)

            ts = []
            for fn in (run_car, run_rccl):
                for _ in range(2):
                    fn()
                torch.cuda.synchronize(dev)
                self.barrier()
                best = float("inf")
                for _ in range(5):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    fn()
                    b.record()
                    b.synchronize()
                    best = min(best, a.elapsed_time(b) * 1000.0)
                ts.append(best)
            tt = torch.tensor(ts, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX, group=self._cpu_group)
            res.append((M, float(tt[0]), float(tt[1])))
        self.check()
        self.rccl_min_rows = rccl_crossover(res)
        self.collective_report = [{"rows": M, "N": N, "car_us": round(tc, 1), "rccl_us": round(tr, 1)}
                                  for M, tc, tr in res]
        return self.collective_report

    def all_gather_lastdim(self, t: torch.Tensor) -> torch.Tensor:
        """[n, V/TP] on every rank -> [n, V] on every rank (in-house IPC gather when
        it fits, else the process group)."""
        if self.world_size == 1:
            return t
        t = t.contiguous()
        car = self.custom_ar
        if car is not None and car.supports_gather(t):
            return car.all_gather(t)
        self._uncapturable("all_gather")
        if t.device.type == "cpu" or self.backend == "gloo":  # gloo: list form
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

    def gather_obj(self, obj):
        """[obj of rank 0, rank 1, ...] on rank 0 (None on the others); CPU group."""
        if self.world_size == 1:
            return [obj]
        out = [None] * self.world_size if self.rank == 0 else None
        dist.gather_object(obj, out, dst=0, group=self._cpu_group)
        return out

    def barrier(self):
        if self.world_size > 1:
            dist.barrier(group=self._cpu_group)

    def max_(self, t: torch.Tensor) -> torch.Tensor:
        """Element-wise maximum over ranks of a small tensor (CPU group: start-up use,
        e.g. per-channel quantisation scales of row-parallel shards)."""
        if self.world_size == 1:
            return t
        c = t.detach().float().cpu().contiguous()
        dist.all_reduce(c, op=dist.ReduceOp.MAX, group=self._cpu_group)
        return c.to(device=t.device, dtype=t.dtype)

    def min_int(self, n: int) -> int:
        """Minimum of a host integer over ranks (CPU group: no device collective)."""
        if self.world_size == 1:
            return n
        t = torch.tensor([n], dtype=torch.long)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self._cpu_group)
        return int(t.item())


def _default_ops(device):
    from ..ops import get_ops

    return get_ops(device)


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
    # bound on any one collective; nothing slow (the first weight download) waits
    # on a collective: weights/hub.py polls a status file instead
    timeout = datetime.timedelta(seconds=float(os.environ.get("HIPSERVE_DIST_TIMEOUT_S", 600)))
    if not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, rank=rank, world_size=ws, timeout=timeout)
    g = TPGroup(rank, ws, dist.group.WORLD, dev)
    g._cpu_group = dist.new_group(backend="gloo", timeout=timeout) if backend != "gloo" else dist.group.WORLD
    g.setup_shm_ring()
    # the custom collectives are created by the ModelRunner once the message sizes
    # (hidden size x token budget, logits shard) are known: ensure_custom_ar()
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
