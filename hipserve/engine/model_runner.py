"""Model runner: owns the model weights, the paged KV cache and the decode
hipGraphs on ONE device (one process per GPU; TP ranks run identical runners).

Per step it turns the scheduler's batch into flat inputs (``StepInputs``, plain
numpy so rank 0 can broadcast it to TP workers), runs the forward, the LM head and
the fused sampling kernel, and returns the sampled ids.

Decode-only batches replay a hipGraph captured per batch-size bucket (the whole
forward + logits + sampling is one graph launch: no per-kernel host launch cost,
SURVEY §3.B step 4); prefill / mixed batches run eagerly.
"""
from __future__ import annotations

import logging
import math
import os
import time
from dataclasses import dataclass, field

import numpy as np
import torch

from ..config import EngineConfig, ModelConfig
from ..models.llama import AttnMeta, LlamaModel
from ..ops import get_ops
from ..parallel.comm import TPGroup
from ..runtime import native
from .scheduler import SchedulerOutput

log = logging.getLogger("hipserve.runner")
PREFILL_TILE = 128
TOP_LOGPROBS = 20   # per-row capacity of the device top-logprobs output (OpenAI max)
GRAPH_BUCKETS = [1, 2, 4, 8, 16, 24, 32, 48, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384, 448, 512]


@dataclass
class StepInputs:
    ids: np.ndarray
    positions: np.ndarray
    slots: np.ndarray
    num_prefill_tokens: int
    num_decode: int
    bt_prefill: np.ndarray | None
    cu_q: np.ndarray | None
    ctx_prefill: np.ndarray | None
    tiles: np.ndarray | None
    bt_decode: np.ndarray | None
    ctx_decode: np.ndarray | None
    logits_rows: np.ndarray
    temperature: np.ndarray
    top_k: np.ndarray
    top_p: np.ndarray
    seeds: np.ndarray
    steps: np.ndarray
    # OpenAI penalties / logprobs, applied on the device (csrc/kernels/penalties.hip)
    pen_slot: np.ndarray | None = None    # int32 [n]: penalty-state slot per sampled row (-1: none)
    pen_vals: np.ndarray | None = None    # float32 [3, n]: presence, frequency, repetition
    nlogprobs: np.ndarray | None = None   # int32 [n]: top-n logprobs wanted per row (0: none)
    pen_init: tuple | None = None         # (slots, off, n_prompt, toks) int32: slots (re)built this step
    top_logprobs: int = 0                 # max n over the rows
    # decode lookahead: per decode row, the row of the PREVIOUS graph step's sampled
    # tokens that is this row's input id (-1: use ids[row]); consumed on the device
    src: np.ndarray | None = None
    extra: dict = field(default_factory=dict)


def pad_table(times: dict, tol: float = 1.03) -> dict:
    """{row count: larger row count to pad it to} from measured GEMM times per row
    count: the fastest count at or above each one, where a larger count must be more
    than ``tol`` faster to be chosen over a smaller one; counts that keep themselves
    are left out."""
    pad, best_t, best_m = {}, float("inf"), None
    for m in sorted(times, reverse=True):
        if times[m] <= best_t * tol:
            best_t, best_m = min(times[m], best_t), m
        pad[m] = best_m
    return {m: p for m, p in pad.items() if p > m}


_PACKED_TIMING: dict = {}  # (prefill units, rows) -> packed vs hipBLASLt timing (ops/pgemm.py tune_packed)


class ModelRunner:
    def __init__(self, ecfg: EngineConfig, mcfg: ModelConfig, tp: TPGroup, device=None):
        self.ecfg = ecfg
        self.mcfg = mcfg
        self.tp = tp
        self.device = torch.device(device or tp.device or ecfg.device)
        if self.device.type == "cuda":
            if self.device.index is None:  # plain "cuda": this process's current device
                self.device = torch.device("cuda", torch.cuda.current_device())
            torch.cuda.set_device(self.device)
        self.dtype = {"bfloat16": torch.bfloat16, "bf16": torch.bfloat16, "auto": torch.bfloat16,
                      "float32": torch.float32, "fp32": torch.float32}[ecfg.dtype]
        if self.device.type == "cuda" and self.dtype != torch.bfloat16:
            raise ValueError("the gfx950 kernels run bf16 activations; use --dtype bfloat16")
        self.ops = get_ops(self.device)
        self.max_model_len = min(ecfg.max_model_len or mcfg.max_position_embeddings,
                                 mcfg.max_position_embeddings)
        self.block_size = ecfg.block_size
        self.model = LlamaModel(mcfg, tp, self.device, self.dtype, self.ops, max_pos=self.max_model_len)
        self.model.decode_partition = ecfg.decode_partition
        self.model.block_size_hint = ecfg.block_size
        if ecfg.kv_fp8:  # e4m3 paged KV cache (the fused qkv -> attention kernel writes bf16 only)
            self.model.kv_dtype = torch.float8_e4m3fn
            self.model.fused_qkv_attention = False
        t0 = time.time()
        self._load_weights()
        self.load_time = time.time() - t0
        from ..utils.faults import FaultInjector

        FaultInjector.from_env().on_init(tp.rank, tp.world_size)  # HIPSERVE_FAULT=rankK:init@0 (tests)
        # start-up breakdown (bench.py reports it: the 70B TP=8 phase must visibly fit its box)
        self.init_times = {"weights_s": round(self.load_time, 2)}
        t1 = time.time()
        if tp.world_size > 1:
            if "tp_exact_reduce" in ecfg.extra:
                tp.exact_reduce = bool(ecfg.extra["tp_exact_reduce"])
            if self.device.type == "cuda":
                # in-house TP collectives sized for the largest message of a step:
                # a prefill chunk's [tokens, hidden] bf16 and the logits shard
                H = mcfg.hidden_size
                msg = max(ecfg.max_num_batched_tokens * H * 2,
                          ecfg.max_num_seqs * self.model.vpad * 2, 8 << 20)
                if tp.ensure_custom_ar(msg):
                    # prefill-sized messages: in-house kernel or RCCL, measured on this node
                    tp.calibrate_collectives(H, ecfg.max_num_batched_tokens)
        self.init_times["collectives_s"] = round(time.time() - t1, 2)
        self.max_bs = min(ecfg.max_num_seqs, max(GRAPH_BUCKETS))
        self.buckets = [b for b in GRAPH_BUCKETS if b <= max(self.max_bs, 1)]
        if self.buckets[-1] < self.max_bs:
            self.buckets.append(self.max_bs)
        # decode-sized messages stay on the in-house collectives, captured or eager
        tp.rccl_floor_rows = max(tp.rccl_floor_rows, self.buckets[-1])
        t1 = time.time()
        # decode GEMM autotune BEFORE the KV pool takes the memory: its cold-weight
        # copies need scratch, and weights whose winner is the packed decode GEMM get
        # their pre-shuffled copy (gemm.PACKED) allocated before the pool is sized
        self.gemm_report = []
        if self.device.type == "cuda" and ecfg.extra.get("gemm_autotune", True):
            from ..ops import gemm

            ms = [b for b in self.buckets if b <= 64]
            self.model.fused_decode = bool(ecfg.extra.get("fused_decode",
                                                          os.environ.get("HIPSERVE_FUSED_DECODE", "1") != "0"))
            fused = self.model.fused_gemm_shapes() if self.model.fused_decode else {}
            self.gemm_report = gemm.TUNER.tune(self.model.gemm_shapes(), self.device, ms, fused=fused)
            self.single_layout = None
            if ecfg.extra.get("packed_decode", True):
                why = self._single_layout_reason()
                if why:  # ONE resident copy per dense weight, in the packed layout
                    n, freed = self.model.to_single_layout()
                    self.single_layout = {"reason": why, "weights": n, "row_major_gb_freed": round(freed / 2**30, 2)}
                else:
                    self.model.pack_decode_weights(gemm.TUNER.packed_shapes())
            # bf16 shadows of quantised weights for hipBLASLt prefill: opt-in (HIPSERVE_QUANT_SHADOW=1
            # or extra quant_dense_shadow). By default a quantised model keeps only its quantised
            # weights (more KV blocks); its prefill dequantises per step into a scratch, which a
            # larger token budget amortises (config.default_batched_tokens)
            shadow = ecfg.extra.get("quant_dense_shadow", os.environ.get("HIPSERVE_QUANT_SHADOW", "0") == "1")
            moes = self.model.quant_moes() if hasattr(self.model, "quant_moes") else []
            if moes and shadow:  # bf16 experts for prefill
                from ..ops import quant as Q

                total = torch.cuda.get_device_properties(self.device).total_memory
                self.quant_shadow_bytes = Q.make_moe_shadows(moes, self.device, (24 << 30) + total // 4)
            qws = self.model.quant_weights() if hasattr(self.model, "quant_weights") else []
            if qws:  # GGUF: split-K of the dequant-MFMA decode GEMM per shape and batch
                from ..ops import quant as Q

                self.gguf_split_report = Q.tune_splits(
                    qws, self.device, [m for m in Q.M_BUCKETS if m <= 64],
                    f8_ms=[m for m in Q.F8_M_BUCKETS if m <= max(64, max(self.buckets, default=1))])
                # GGUF prefill: the block kernel or dequant + hipBLASLt per shape, timed at the
                # token budget (the LM head only sees a few rows per prefill: not timed)
                lm = getattr(self.model, "lm_head", None)
                self.qprefill_report = Q.tune_qprefill([w for w in qws if w is not lm], self.device,
                                                       min(ecfg.max_num_batched_tokens, 8192)) \
                    if Q.QPREFILL_MODE == "auto" else []
                total = torch.cuda.get_device_properties(self.device).total_memory
                self.quant_shadow_bytes = getattr(self, "quant_shadow_bytes", 0)
                if shadow:
                    gguf = ecfg.extra.get("gguf_dense_shadow", shadow)
                    self.quant_shadow_bytes += Q.make_dense_shadows(qws, self.device, (24 << 30) + total // 4,
                                                                    gguf=gguf)
                # FP8: which projections prefill on hipBLASLt's FP8 GEMM (a per-call
                # re-layout of the tiled copy by default, ops/quant.py FP8_LIB)
                self.quant_shadow_bytes += Q.make_fp8_plain(qws, self.device, (24 << 30) + total // 4)
            if getattr(self.mcfg, "num_experts", 0) and hasattr(self.model, "tune_moe_prefill"):
                # MoE prefill expert GEMMs: hipBLASLt grouped vs the packed one-launch kernel
                self.moe_prefill_report = self.model.tune_moe_prefill(min(ecfg.max_num_batched_tokens, 16384))
            torch.cuda.empty_cache()
        self.init_times["decode_gemm_tune_s"] = round(time.time() - t1, 2)
        t1 = time.time()
        # (TunableOp solution choice for the prefill GEMMs was measured no faster than the
        # heuristic on sustained prefill chains, profiles/r1_prefill_gemm_tunableop.md, and
        # the bf16 prefill_gemm.hip kernels lost to hipBLASLt everywhere: both removed)
        # ragged prefill chunks: hipBLASLt's heuristic picks slower kernels for some
        # token counts (Llama-3-8B: the 4-projection chain takes 21.7 ms at 7,393 rows
        # vs 18.8 ms at 8,192, tools/bench_prefill_m.py); rank 0 times the model's
        # prefill GEMMs per 256-row count once and pads a chunk to the fastest count at
        # or above it (padding rows: token 0, no KV write, outputs unused)
        self.prefill_pad = None
        if self.device.type == "cuda" and ecfg.extra.get("prefill_pad", True) and tp.rank == 0:
            self.prefill_pad = self._probe_prefill_pad()
        # device penalty state: one slot per concurrently running sequence (a slot is
        # held from the first sample to finish / abort / preemption), so a slot is
        # always free for a running sequence: max_num_seqs x V x ~4.1 B (512 slots of a
        # 128K vocabulary: 270 MB of 288 GB)
        V = mcfg.vocab_size
        nslots = max(1, ecfg.max_num_seqs)
        self.pen_counts = torch.zeros(nslots, V, dtype=torch.int32, device=self.device)
        self.pen_seen = torch.zeros(nslots, (V + 31) // 32, dtype=torch.int32, device=self.device)
        self._free_pen = list(range(nslots - 1, -1, -1))
        self.init_times["pad_probe_s"] = round(time.time() - t1, 2)
        t1 = time.time()
        self.num_blocks = self._num_kv_blocks()
        self.kv = self.model.allocate_kv_cache(self.num_blocks, self.block_size)
        self.init_times["kv_alloc_s"] = round(time.time() - t1, 2)
        self.pad_block = self.num_blocks - 1          # scratch block for graph padding rows
        self.width = -(-self.max_model_len // self.block_size)
        part = ecfg.decode_partition
        self.max_parts = -(-self.width * self.block_size // part)
        nq = self.model.nq
        self.tmp_out = torch.empty(self.max_bs, nq, self.max_parts, mcfg.head_dim,
                                   device=self.device, dtype=torch.float32)
        self.tmp_ml = torch.empty(self.max_bs, nq, self.max_parts, 2, device=self.device,
                                  dtype=torch.float32)
        self.stats = {"graph_steps": 0, "eager_steps": 0}  # which path each step took
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self.graph_pool = None
        self._static = None
        self.use_graphs = self.device.type == "cuda" and not ecfg.enforce_eager
        if self.use_graphs:
            self._capture_graphs()
        self.init_times["graph_capture_s"] = round(getattr(self, "graph_capture_time", 0.0), 2)
        # every rank's breakdown on rank 0 (a TP pod's start-up is as slow as its slowest rank)
        self.init_times_ranks = tp.gather_obj(dict(self.init_times))

    # ------------------------------------------------------------ setup
    def _load_weights(self):
        fmt = self.ecfg.load_format
        model = self.ecfg.model
        if fmt == "auto":
            from ..config import PRESETS

            key = model.lower().split("/")[-1]
            if key in PRESETS:
                fmt = "dummy"
            elif model.endswith(".gguf"):
                fmt = "gguf"
            else:
                fmt = "safetensors"
        quant = self.ecfg.extra.get("quantization")
        if fmt == "dummy" and quant:
            self.model.allocate_random_quant(quant, seed=self.ecfg.seed)
        elif fmt == "dummy":
            self.model.allocate_random(seed=self.ecfg.seed)
        elif fmt == "safetensors":
            from ..weights.safetensors_loader import load_hf_weights

            load_hf_weights(self.model, model)
        elif fmt == "gguf":
            from ..weights.gguf import load_gguf_weights

            load_gguf_weights(self.model, model)
        else:
            raise ValueError(f"unknown load_format {fmt}")
        self.load_format = fmt

    def _single_layout_reason(self) -> str | None:
        """Whether the dense projections keep ONLY their packed copy (``gemm.PackedLinear``).
        HIPSERVE_SINGLE_LAYOUT=1 forces it, 0 keeps row-major + packed copies; ``auto``
        (default): single when the two copies would not leave 24 GiB + a quarter of HBM
        for the KV cache (e.g. Llama-3-70B on one MI355X), or when the packed prefill GEMM
        times at least as fast as hipBLASLt on this model's prefill units."""
        mode = os.environ.get("HIPSERVE_SINGLE_LAYOUT", self.ecfg.extra.get("single_layout", "auto"))
        m = self.model
        if str(mode) == "0" or not hasattr(m, "single_layout_ok") or not m.single_layout_ok():
            return None
        if str(mode) == "1":
            return "forced"
        from ..ops import gemm, pgemm

        lw = m.layers[0]
        ws = [w for w in (lw.wqkv, lw.wo, lw.wgu, lw.wd) if isinstance(w, torch.Tensor)]
        per_layer = sum(w.numel() * w.element_size() for w in ws if gemm.packable(*w.shape))
        need = per_layer * len(m.layers)
        free, total = torch.cuda.mem_get_info(self.device)
        # TP ranks decide together (min over ranks): ranks with different weight layouts
        # would run different prefill GEMMs and round differently
        margin = (free - need - (24 << 30) - total // 4) >> 20  # MiB
        if self.tp.world_size > 1:
            margin = self.tp.min_int(int(margin))
        if margin < 0:
            return "memory"
        units = []
        for kind, w in (("plain", lw.wqkv), ("add", lw.wo), ("glu", lw.wgu), ("add", lw.wd)):
            if isinstance(w, torch.Tensor) and gemm.packable(*w.shape) and (kind != "glu" or w.shape[0] % 128 == 0):
                units.append((kind, w.shape[0], w.shape[1]))
        M = self.ecfg.max_num_batched_tokens
        # TP: the o / down epilogue is the cross-rank norm; small token budgets: prefill
        # GEMMs are not the bottleneck (and every engine of a test process decides alike)
        if not units or self.tp.world_size > 1 or M < 2048:
            return None
        key = (tuple(units), M)
        r = _PACKED_TIMING.get(key)
        if r is None:  # one timing per shape set and process (engines in one process agree),
            # and per device / kernel build across starts (ops/tune_cache.py)
            from ..ops import tune_cache as TC

            r = TC.get(self.device, "packed_prefill", [units, M])
            if r is None:
                r = pgemm.tune_packed(units, M, self.device, self.ops)
                TC.put(self.device, "packed_prefill", [units, M], r)
                TC.flush()
            _PACKED_TIMING[key] = r
        self.packed_prefill_report = r
        return "prefill timing" if r["packed_ms"] <= r["blas_ms"] else None

    def _num_kv_blocks(self) -> int:
        if self.ecfg.num_kv_blocks:
            return int(self.ecfg.num_kv_blocks)
        per_block = self.model.kv_bytes_per_block(self.block_size)
        if self.device.type != "cuda":
            want = max(64, 4 * self.max_model_len // self.block_size)
            return min(want, 4096)
        torch.cuda.synchronize(self.device)
        free, total = torch.cuda.mem_get_info(self.device)
        used = total - free
        H, I = self.mcfg.hidden_size, self.model.inter
        T = self.ecfg.max_num_batched_tokens
        qkv = (self.model.nq + 2 * self.model.nkv) * self.mcfg.head_dim
        act = T * (2 * I + I + qkv + 6 * H) * 2 * 2
        logits = self.ecfg.max_num_seqs * self.mcfg.vocab_size * 4 * 3
        work = self.ecfg.max_num_seqs * self.model.nq * (
            -(-self.max_model_len // self.ecfg.decode_partition)) * (self.mcfg.head_dim + 2) * 4
        reserve = act + logits + work + (2 << 30)
        budget = total * self.ecfg.gpu_memory_utilization - used - reserve
        n = int(budget // per_block)
        if n < 16:
            raise RuntimeError(f"not enough GPU memory for the KV cache (budget {budget / 2**30:.1f} GiB)")
        # all TP ranks must agree on the pool size
        return self.tp.min_int(n)

    def _probe_prefill_pad(self) -> dict | None:
        """{rows rounded up to 256: the row count (>= it, <= the token budget) whose
        prefill GEMM chain (qkv, o, gate|up, down of one layer, hipBLASLt) is fastest};
        None for models whose prefill is not four dense bf16 projections (MoE, quantised)."""
        import torch.nn.functional as F

        layers = getattr(self.model, "layers", None)
        if not layers or any(getattr(lw, "router", None) is not None for lw in layers):
            return None
        lw = layers[0]
        ws = [getattr(lw, n, None) for n in ("wqkv", "wo", "wgu", "wd")]
        if not all(isinstance(w, torch.Tensor) and w.dim() == 2 and w.dtype == torch.bfloat16 for w in ws):
            return None
        budget = self.ecfg.max_num_batched_tokens
        ms = list(range(1024, budget + 1, 256))
        if len(ms) < 2:
            return None
        from ..ops import tune_cache as TC

        ck = [[list(w.shape) for w in ws], budget]
        hit = TC.get(self.device, "prefill_pad", ck)
        if hit is not None:  # timed by a previous start on this device and kernel build
            times = {int(m): t for m, t in hit.items()}
            self.prefill_pad_times = {m: round(t / 2, 3) for m, t in times.items()}
            return pad_table(times)
        x = torch.randn(budget, max(w.shape[1] for w in ws), device=self.device, dtype=torch.bfloat16)

        def chain(m):
            for w in ws:
                F.linear(x[:m, :w.shape[1]], w)

        times = {}
        for m in ms:
            chain(m)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(2):
                chain(m)
            e1.record()
            e1.synchronize()
            times[m] = e0.elapsed_time(e1)
        del x
        TC.put(self.device, "prefill_pad", ck, times)
        TC.flush()
        self.prefill_pad_times = {m: round(t / 2, 3) for m, t in times.items()}
        return pad_table(times)

    def _pad_rows(self, T: int) -> int:
        if not self.prefill_pad or T < 1024:
            return T
        return self.prefill_pad.get(-(-T // 256) * 256, T)

    @property
    def usable_blocks(self) -> int:
        return self.num_blocks - 1

    # ------------------------------------------------------------ inputs
    def prepare(self, so: SchedulerOutput) -> StepInputs:
        """Flatten a scheduled batch (rank 0)."""
        rt = native()
        bs = self.block_size
        seqs = so.prefill + so.decode
        tables = [s.seq.block_ids for s in seqs]
        starts = [s.start for s in seqs]
        ends = [s.end for s in seqs]
        bt, slots, pos = rt.build_batch(tables, starts, ends, bs, self.width)
        np_ = len(so.prefill)
        ids = np.empty(len(slots), dtype=np.int64)
        t = 0
        for s in seqs:
            q = s.seq
            if s.num_tokens == 1:
                ids[t] = q.token_at(s.start)
            else:
                npt = q.num_prompt_tokens
                if s.end <= npt:
                    ids[t:t + s.num_tokens] = q.prompt_token_ids[s.start:s.end]
                else:
                    ids[t:t + s.num_tokens] = q.all_token_ids()[s.start:s.end]
            t += s.num_tokens
        if np_ and not any(s.seq.mm is not None for s in seqs):
            Tpad = self._pad_rows(len(ids))
            if Tpad > len(ids):  # padding rows: token 0 at position 0, no KV write
                extra = Tpad - len(ids)
                ids = np.concatenate([ids, np.zeros(extra, np.int64)])
                pos = np.concatenate([pos, np.zeros(extra, pos.dtype)])
                slots = np.concatenate([slots, np.full(extra, -1, slots.dtype)])
                self.stats["padded_rows"] = self.stats.get("padded_rows", 0) + extra
        Tp = sum(s.num_tokens for s in so.prefill)
        rows = []
        t = 0
        sample_seqs = []
        for s in so.prefill:
            t += s.num_tokens
            if s.samples:
                rows.append(t - 1)
                sample_seqs.append(s.seq)
        for j, s in enumerate(so.decode):
            rows.append(Tp + j)
            sample_seqs.append(s.seq)
        cu_q = ctx_p = tiles = bt_p = None
        if np_:
            cu = np.zeros(np_ + 1, dtype=np.int32)
            cu[1:] = np.cumsum([s.num_tokens for s in so.prefill])
            cu_q = cu
            ctx_p = np.array([s.end for s in so.prefill], dtype=np.int32)
            # heaviest (latest absolute position) first: the prefill attention kernel
            # dispatches tiles in this order (longest-processing-time against the causal tail)
            tl = sorted(((i, r) for i, s in enumerate(so.prefill) for r in range(0, s.num_tokens, PREFILL_TILE)),
                        key=lambda t: so.prefill[t[0]].end - so.prefill[t[0]].num_tokens + t[1], reverse=True)
            tiles = np.array(tl, dtype=np.int32).reshape(-1, 2)
            bt_p = bt[:np_]
        bt_d = ctx_d = None
        if so.decode:
            bt_d = bt[np_:]
            ctx_d = np.array([s.end for s in so.decode], dtype=np.int32)
        n = len(sample_seqs)
        n_pf = len(sample_seqs) - len(so.decode)  # rows sampling after a (last) prefill chunk
        temp = np.empty(n, np.float32)
        topk = np.empty(n, np.int32)
        topp = np.empty(n, np.float32)
        seeds = np.empty(n, np.int64)
        steps = np.empty(n, np.int64)
        pen_slot = pen_vals = nlp = pen_init = None
        topn = 0
        init = []
        for i, q in enumerate(sample_seqs):
            p = q.params
            temp[i] = p.temperature
            topk[i] = p.top_k if p.top_k > 0 else 0
            topp[i] = p.top_p
            seeds[i] = q.seed
            steps[i] = len(q.output_token_ids)
            if p.has_penalties:
                if pen_slot is None:
                    pen_slot = np.full(n, -1, np.int32)
                    pen_vals = np.zeros((3, n), np.float32)
                    pen_vals[2] = 1.0
                if q.pen_slot is None:
                    q.pen_slot = self._free_pen.pop()
                pen_slot[i] = q.pen_slot
                pen_vals[:, i] = (p.presence_penalty, p.frequency_penalty, p.repetition_penalty)
                if i < n_pf:  # first sample (or a recompute): rebuild the slot from the ids so far
                    init.append(q)
            if p.logprobs:
                if nlp is None:
                    nlp = np.zeros(n, np.int32)
                nlp[i] = min(p.logprobs, TOP_LOGPROBS)
                topn = max(topn, int(nlp[i]))
        if init:
            ids_l = [q.prompt_token_ids + [t for t in q.output_token_ids if t >= 0] for q in init]
            off = np.zeros(len(init) + 1, np.int32)
            off[1:] = np.cumsum([len(x) for x in ids_l])
            pen_init = (np.array([q.pen_slot for q in init], np.int32), off,
                        np.array([q.num_prompt_tokens for q in init], np.int32),
                        np.fromiter((t for x in ids_l for t in x), np.int32, int(off[-1])))
        inp = StepInputs(ids, pos, slots, Tp, len(so.decode), bt_p, cu_q, ctx_p, tiles, bt_d, ctx_d,
                         np.array(rows, dtype=np.int64), temp, topk, topp, seeds, steps,
                         pen_slot, pen_vals, nlp, pen_init, topn)
        if any(s.seq.mm is not None for s in seqs):
            self._prepare_mm(seqs, inp)
        return inp

    def _prepare_mm(self, seqs, inp: StepInputs):
        """Multimodal rows of a batch: rotary positions of the sequences' tokens from
        their MRoPE tables (prompt) or index + delta (generated tokens); the image
        tokens, whose three axes differ, get their own table rows; each image whose
        token span intersects a prefill chunk is listed with the chunk's slice of it
        (every TP rank runs the replicated vision tower on the same pixels)."""
        pos = np.array(inp.positions, dtype=np.int64, copy=True)
        rope_rows, rope_pos, images = [], [], []
        t = 0
        for s in seqs:
            mm = s.seq.mm
            n = s.num_tokens
            if mm is not None:
                npr = s.seq.num_prompt_tokens
                a, b = s.start, min(s.end, npr)
                if a < b:
                    p3 = mm.pos3[:, a:b]
                    pos[t:t + b - a] = p3[0]
                    odd = np.nonzero((p3[0] != p3[1]) | (p3[0] != p3[2]))[0]
                    if odd.size:
                        rope_rows.append(odd + t)
                        rope_pos.append(p3[:, odd])
                    for (ia, ib), im in zip(mm.spans, mm.images):
                        lo, hi = max(ia, a), min(ib, b)
                        if lo < hi:
                            images.append((t + lo - a, lo - ia, hi - ia, im.pixels, tuple(im.grid), im.digest))
                if s.end > npr:
                    k0 = max(s.start, npr)
                    pos[t + k0 - s.start:t + n] = np.arange(k0, s.end) + mm.delta
            t += n
        inp.positions = pos
        if rope_rows or images:
            inp.extra["mm"] = {
                "rope_rows": np.concatenate(rope_rows) if rope_rows else np.zeros(0, np.int64),
                "rope_pos": np.concatenate(rope_pos, 1) if rope_pos else np.zeros((3, 0), np.int64),
                "images": images}

    def release(self, seq):
        """A finished / aborted sequence gives its penalty slot back."""
        if seq.pen_slot is not None:
            self._free_pen.append(seq.pen_slot)
            seq.pen_slot = None

    # ------------------------------------------------------------ execution
    def _t(self, a, dtype=None):
        if a is None:
            return None
        t = torch.from_numpy(np.ascontiguousarray(a))
        if self.device.type == "cuda":
            t = t.pin_memory().to(self.device, non_blocking=True)
        return t

    @property
    def max_graph_batch(self) -> int:
        return self.buckets[-1] if self.use_graphs else 0

    def graph_eligible(self, inp: StepInputs) -> bool:
        # penalties and logprobs run inside the graph (device state + per-row inputs)
        return (self.use_graphs and inp.num_prefill_tokens == 0 and inp.pen_init is None
                and 0 < inp.num_decode <= self.buckets[-1])

    @torch.inference_mode()
    def execute(self, inp: StepInputs):
        """Returns (tokens np.int64 [n], logprobs np.float32 [n], top_logprobs or None)."""
        n = len(inp.logits_rows)
        if self.graph_eligible(inp):
            return self.wait(self.launch(inp))
        if inp.src is not None:
            raise RuntimeError("device-side input ids (lookahead) need the hipGraph decode path")
        self.stats["eager_steps"] += 1
        ids = self._t(inp.ids)
        meta = AttnMeta(
            num_prefill_tokens=inp.num_prefill_tokens, num_decode=inp.num_decode,
            positions=self._t(inp.positions), slot_mapping=self._t(inp.slots),
            bt_prefill=self._t(inp.bt_prefill), cu_q=self._t(inp.cu_q),
            ctx_prefill=self._t(inp.ctx_prefill), tiles=self._t(inp.tiles),
            bt_decode=self._t(inp.bt_decode), ctx_decode=self._t(inp.ctx_decode),
            tmp_out=self.tmp_out, tmp_ml=self.tmp_ml)
        if inp.num_decode > self.max_bs:
            meta.tmp_out = torch.empty(inp.num_decode, *self.tmp_out.shape[1:], device=self.device)
            meta.tmp_ml = torch.empty(inp.num_decode, *self.tmp_ml.shape[1:], device=self.device)
        if "mm" in inp.extra:
            self._attach_mm(inp.extra["mm"], meta, len(inp.ids))
        hidden = self.model.forward(ids, meta, self.kv)
        if n == 0:
            return np.zeros(0, np.int64), np.zeros(0, np.float32), None
        rows = self._t(inp.logits_rows)
        logits = self.model.compute_logits(hidden.index_select(0, rows))
        top = None
        if inp.top_logprobs:  # raw (pre-penalty) log-probs, as vLLM's default mode
            ti = torch.empty(n, TOP_LOGPROBS, dtype=torch.int32, device=self.device)
            tl = torch.empty(n, TOP_LOGPROBS, dtype=torch.float32, device=self.device)
            self.ops.top_logprobs(logits, self._t(inp.nlogprobs), ti, tl)
        pslot = None
        if inp.pen_slot is not None:
            if inp.pen_init is not None:
                self.ops.penalty_init(self.pen_counts, self.pen_seen, *[self._t(a) for a in inp.pen_init])
            pslot = self._t(inp.pen_slot)
            pv = self._t(inp.pen_vals)
            self.ops.penalty_apply(logits, pslot, pv[0], pv[1], pv[2], self.pen_counts, self.pen_seen)
        tok = torch.empty(n, dtype=torch.long, device=self.device)
        lp = torch.empty(n, dtype=torch.float32, device=self.device)
        self.ops.sample(tok, lp, logits, self._t(inp.temperature), self._t(inp.top_k),
                        self._t(inp.top_p), self._t(inp.seeds), self._t(inp.steps))
        if pslot is not None:
            self.ops.penalty_update(tok, pslot, self.pen_counts, self.pen_seen)
        if inp.top_logprobs:
            top = (ti.cpu().numpy(), tl.cpu().numpy())
        return tok.cpu().numpy(), lp.cpu().numpy(), top

    def _attach_mm(self, mm: dict, meta: AttnMeta, T: int):
        """Vision-tower outputs and MRoPE rows of a multimodal prefill batch into the
        attention metadata: a per-row rotary table (the model's table gathered at the
        rows' positions, image rows replaced by their 3D MRoPE rows) with
        positions = row index, and the image embeddings / DeepStack features with the
        batch rows they belong to."""
        from ..models.vision import image_geometry
        from ..multimodal import mrope_cos_sin

        cfg = self.mcfg
        if len(mm["rope_rows"]):
            cs = self.model.cos_sin.index_select(0, meta.positions)
            rows = self._t(mm["rope_rows"])
            vals = mrope_cos_sin(mm["rope_pos"], cfg.head_dim, cfg.rope_theta, cfg.mrope_section)
            cs.index_copy_(0, rows, self._t(vals))
            meta.cos_sin = cs
            meta.positions = torch.arange(T, device=self.device)
        if not mm["images"]:
            return
        vis = self.model.visual
        # every distinct image of the step goes through the tower in ONE forward (one
        # attention segment per frame): one GEMM per projection for all of them
        uniq = {}
        for _, _, _, pixels, grid, digest in mm["images"]:
            uniq.setdefault(digest, (pixels, grid))
        geo = image_geometry([g for _, g in uniq.values()], vis.cfg)
        emb, ds_all = vis.forward(torch.from_numpy(np.concatenate([p for p, _ in uniq.values()])), geo)
        cache, off = {}, 0
        m2 = vis.cfg.spatial_merge_size ** 2
        for digest, (pixels, _) in uniq.items():
            n = pixels.shape[0] // m2
            cache[digest] = (emb[off:off + n], [d[off:off + n] for d in ds_all])
            off += n
        rows, embs, dss = [], [], []
        for row0, lo, hi, pixels, grid, digest in mm["images"]:
            e, ds = cache[digest]
            rows.append(torch.arange(row0, row0 + hi - lo))
            embs.append(e[lo:hi])
            dss.append([d[lo:hi] for d in ds])
        meta.mm_rows = torch.cat(rows).to(self.device)
        meta.mm_embeds = torch.cat(embs).to(self.model.dtype)
        meta.mm_deepstack = [torch.cat([d[j] for d in dss]).to(self.model.dtype) for j in range(len(dss[0]))]

    # ------------------------------------------------------------ hipGraphs
    def _graph_forward(self, b: int, full: bool = True):
        """The captured decode step. The lean variant (``full=False``) leaves out the
        OpenAI penalty and top-n logprob kernels and the sampler's second threshold
        round (needed only by rows that combine top-k with top-p); a step whose rows
        need none of them replays it: five launches fewer, ~35 us of a ~5.4 ms
        Llama-3-8B step."""
        st = self._static
        meta = AttnMeta(num_prefill_tokens=0, num_decode=b, positions=st["pos"][:b],
                        slot_mapping=st["slots"][:b], bt_decode=st["bt"][:b], ctx_decode=st["ctx"][:b],
                        tmp_out=self.tmp_out, tmp_ml=self.tmp_ml)
        # lookahead ids: resolved inside the model's first kernel when it can
        # (embed_rmsnorm), else by the model's id select (LlamaModel.resolve_ids)
        meta.id_src = (st["src"][:b], st["tok"])
        hidden = self.model.forward(st["ids"][:b], meta, self.kv)
        logits = self.model.compute_logits(hidden)
        # penalties / top-n logprobs: early-exit kernels for rows that want none; top-n
        # log-probs of the raw (pre-penalty) distribution, as vLLM's default mode
        if full:
            self.ops.top_logprobs(logits, st["nlp"][:b], st["top_ids"][:b], st["top_lp"][:b])
            self.ops.penalty_apply(logits, st["pslot"][:b], st["pres"][:b], st["freq"][:b], st["rep"][:b],
                                   self.pen_counts, self.pen_seen)
        self.ops.sample(st["tok"][:b], st["lp"][:b], logits, st["temp"][:b], st["topk"][:b],
                        st["topp"][:b], st["seeds"][:b], st["steps"][:b], two_rounds=full)
        if full:
            self.ops.penalty_update(st["tok"][:b], st["pslot"][:b], self.pen_counts, self.pen_seen)

    def _stage_in(self, b: int, sg):
        """Pinned staging set -> device static inputs, one zero-copy dispatch
        (csrc/kernels/stage_copy.hip); captured at the head of a parity graph."""
        st, mb, W = self._static, self.buckets[-1], self.width
        torch.ops.hipserve.stage_copy([st["d64"], st["d32"][: b * W], st["d32"][mb * W:], st["df"]],
                                      [sg["h64"], sg["h32"][: b * W], sg["h32"][mb * W:], sg["hf"]],
                                      self.device.index or 0)

    def _stage_out(self, b: int, sg):
        st = self._static
        torch.ops.hipserve.stage_copy([sg["tok"][:b], sg["lp"][:b], sg["top_ids"][:b], sg["top_lp"][:b]],
                                      [st["tok"][:b], st["lp"][:b], st["top_ids"][:b], st["top_lp"][:b]],
                                      self.device.index or 0)

    @torch.inference_mode()
    def _capture_graphs(self):
        mb, W, dev = self.buckets[-1], self.width, self.device
        # host staging (pinned, double-buffered by launch parity so step k+1 can be
        # staged while step k runs) and device static buffers, one region per dtype
        self._stage = []
        for _ in range(2):
            self._stage.append({
                "h64": torch.zeros(6 * mb, dtype=torch.long).pin_memory(),
                "h32": torch.zeros(mb * W + 4 * mb, dtype=torch.int32).pin_memory(),
                "hf": torch.zeros(5 * mb, dtype=torch.float32).pin_memory(),
                "tok": torch.zeros(mb, dtype=torch.long).pin_memory(),
                "lp": torch.zeros(mb, dtype=torch.float32).pin_memory(),
                "top_ids": torch.zeros(mb, TOP_LOGPROBS, dtype=torch.int32).pin_memory(),
                "top_lp": torch.zeros(mb, TOP_LOGPROBS, dtype=torch.float32).pin_memory(),
                "done": None,
            })
        self._launches = 0
        # HIPSERVE_STAGE_COPY=blit: per-buffer hipMemcpyAsync instead of the staging kernel
        self._stage_kernel = os.environ.get("HIPSERVE_STAGE_COPY", "kernel") != "blit"
        d64 = torch.zeros(6 * mb, dtype=torch.long, device=dev)
        d32 = torch.zeros(mb * W + 4 * mb, dtype=torch.int32, device=dev)
        df = torch.zeros(5 * mb, dtype=torch.float32, device=dev)
        st = {
            "d64": d64, "d32": d32, "df": df,
            "ids": d64[0:mb], "pos": d64[mb:2 * mb], "slots": d64[2 * mb:3 * mb],
            "seeds": d64[3 * mb:4 * mb], "steps": d64[4 * mb:5 * mb], "src": d64[5 * mb:6 * mb],
            "bt": d32[: mb * W].view(mb, W), "ctx": d32[mb * W: mb * W + mb],
            "topk": d32[mb * W + mb: mb * W + 2 * mb],
            "pslot": d32[mb * W + 2 * mb: mb * W + 3 * mb], "nlp": d32[mb * W + 3 * mb: mb * W + 4 * mb],
            "temp": df[0:mb], "topp": df[mb:2 * mb],
            "pres": df[2 * mb:3 * mb], "freq": df[3 * mb:4 * mb], "rep": df[4 * mb:5 * mb],
            "tok": torch.zeros(mb, dtype=torch.long, device=dev),
            "lp": torch.zeros(mb, dtype=torch.float32, device=dev),
            "top_ids": torch.zeros(mb, TOP_LOGPROBS, dtype=torch.int32, device=dev),
            "top_lp": torch.zeros(mb, TOP_LOGPROBS, dtype=torch.float32, device=dev),
        }
        self._static = st
        st["bt"].fill_(self.pad_block)
        st["ctx"].fill_(1)
        st["slots"].fill_(self.pad_block * self.block_size)
        st["topp"].fill_(1.0)
        st["src"].fill_(-1)
        st["pslot"].fill_(-1)
        st["rep"].fill_(1.0)
        t0 = time.time()
        # TP ranks enter the captured collectives together (the tuner and the
        # weight packing take different times per rank; a custom-collective
        # barrier must not spin through a peer's whole setup)
        self.tp.barrier()
        # every bucket and variant runs eagerly once, on the stream the graphs are then
        # captured on, before any capture starts: a library's first-use work for a shape
        # (hipBLASLt's workspace / code-object load, a lazily built table) must never
        # happen under capture. Which shapes reach hipBLASLt at decode depends on the
        # tuner's per-box timing or on a tuning-cache hit (round 5's TP=2 capture abort:
        # 'operation not permitted when stream is capturing' from hipBLASLt), so warming
        # only the largest bucket was not enough
        stream = torch.cuda.Stream(device=dev)
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):
            self._graph_forward(self.buckets[-1])
            for b in reversed(self.buckets):
                for full in (True, False):
                    self._graph_forward(b, full)
        stream.synchronize()
        torch.cuda.synchronize(dev)
        self.tp.barrier()
        self.graph_pool = torch.cuda.graph_pool_handle()
        for b in reversed(self.buckets):
            # staging kernel: one graph per staging-set parity with the H2D and D2H
            # copies captured inside, so consecutive steps are back-to-back graphs
            # (a standalone dispatch after a graph waits ~0.2 ms for the graph's end)
            for par in ((0, 1) if self._stage_kernel else (None,)):
                for full in (True, False):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=self.graph_pool, stream=stream):
                        if par is not None:
                            self._stage_in(b, self._stage[par])
                        self._graph_forward(b, full)
                        if par is not None:
                            self._stage_out(b, self._stage[par])
                    self.graphs[(b, par, full)] = g
        torch.cuda.synchronize(dev)
        self.graph_capture_time = time.time() - t0

    @torch.inference_mode()
    def launch(self, inp: StepInputs):
        """Stage inputs and replay the decode hipGraph WITHOUT waiting; the sampled
        ids are copied into pinned host memory behind the graph. Returns a handle
        for ``wait``. Safe to call again before waiting (parity double buffer)."""
        n = inp.num_decode
        b = next(x for x in self.buckets if x >= n)
        mb, W = self.buckets[-1], self.width
        self.stats["graph_steps"] += 1
        sg = self._stage[self._launches & 1]
        self._launches += 1
        if sg["done"] is not None:
            sg["done"].synchronize()  # the launch two steps ago read this staging set
        h64, h32, hf = sg["h64"], sg["h32"], sg["hf"]
        pad_slot = self.pad_block * self.block_size
        a64 = h64.numpy()
        a64[0:n] = inp.ids
        a64[n:b] = 0
        a64[mb:mb + n] = inp.positions
        a64[mb + n:mb + b] = 0
        a64[2 * mb:2 * mb + n] = inp.slots
        a64[2 * mb + n:2 * mb + b] = pad_slot
        a64[3 * mb:3 * mb + n] = inp.seeds
        a64[4 * mb:4 * mb + n] = inp.steps
        if inp.src is not None:
            a64[5 * mb:5 * mb + n] = inp.src
        else:
            a64[5 * mb:5 * mb + n] = -1
        a64[5 * mb + n:5 * mb + b] = -1
        a32 = h32.numpy()
        btv = a32[: mb * W].reshape(mb, W)
        btv[:n] = inp.bt_decode
        btv[n:b] = self.pad_block
        a32[mb * W: mb * W + n] = inp.ctx_decode
        a32[mb * W + n: mb * W + b] = 1
        a32[mb * W + mb: mb * W + mb + n] = inp.top_k
        o = mb * W + 2 * mb  # penalty slots, then top-n logprobs counts
        a32[o:o + n] = inp.pen_slot if inp.pen_slot is not None else -1
        a32[o + n:o + b] = -1
        a32[o + mb:o + mb + n] = inp.nlogprobs if inp.nlogprobs is not None else 0
        a32[o + mb + n:o + mb + b] = 0
        af = hf.numpy()
        af[0:n] = inp.temperature
        af[n:b] = 0.0
        af[mb:mb + n] = inp.top_p
        if inp.pen_vals is not None:
            af[2 * mb:2 * mb + n] = inp.pen_vals[0]
            af[3 * mb:3 * mb + n] = inp.pen_vals[1]
            af[4 * mb:4 * mb + n] = inp.pen_vals[2]
        else:
            af[2 * mb:2 * mb + n] = 0.0
            af[3 * mb:3 * mb + n] = 0.0
            af[4 * mb:4 * mb + n] = 1.0
        st = self._static
        full = (inp.pen_slot is not None or inp.nlogprobs is not None
                or bool(np.any((inp.top_k[:n] > 0) & (inp.top_p[:n] < 1.0))))
        if self._stage_kernel:  # the graph of this parity stages in/out itself
            self.graphs[(b, (self._launches - 1) & 1, full)].replay()
        else:
            st["d64"].copy_(h64, non_blocking=True)
            st["d32"][: b * W].copy_(h32[: b * W], non_blocking=True)
            st["d32"][mb * W:].copy_(h32[mb * W:], non_blocking=True)
            st["df"].copy_(hf, non_blocking=True)
            self.graphs[(b, None, full)].replay()
            for k in ("tok", "lp", "top_ids", "top_lp"):
                sg[k][:n].copy_(st[k][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        sg["done"] = ev
        return (sg, n, ev, inp.top_logprobs)

    def wait(self, handle):
        """(tokens, logprobs, top-n (ids, logprobs) or None) of a launched step."""
        sg, n, ev, topn = handle
        ev.synchronize()
        top = (sg["top_ids"][:n].numpy().copy(), sg["top_lp"][:n].numpy().copy()) if topn else None
        return sg["tok"][:n].numpy().copy(), sg["lp"][:n].numpy().copy(), top
