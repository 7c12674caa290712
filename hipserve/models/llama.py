"""Decoder-only transformer families on the hipserve op set (SURVEY §3.F hot loop):
Llama-2/3, TinyLlama, Mistral-style GQA, Mixtral MoE, Qwen2 (qkv bias), Qwen3
(per-head q/k RMSNorm), Qwen3-MoE (128 experts, top-8), Gemma-3 text (GeGLU,
sandwich norms, embedding scale, interleaved sliding-window / global layers with
their own RoPE bases) and Phi-3 — one parameterised model, the family switches
are ``ModelConfig`` fields (the reference's chart defaults are Gemma-3, Qwen3-VL-MoE
and Qwen3: vllm-models/helm-chart/values.yaml:1-19).

Per layer: fused add+RMSNorm -> merged QKV GEMM (hipBLASLt) -> fused RoPE +
paged-cache write -> paged attention (prefill and/or decode kernels) -> o_proj GEMM
-> TP all-reduce -> fused add+RMSNorm -> merged gate/up GEMM -> SiLU*up ->
down GEMM -> TP all-reduce. Weights are held as plain tensors already laid out
for the kernels ([out, in] row-major, TP-sharded on load), no nn.Module tracing.

The reference never contains model code — it runs `vllm/vllm-openai:v0.11.0`
with `--tensor-parallel-size <gpuRequestCount>`
(vllm-models/helm-chart/templates/model-deployments.yaml:26-39); this is the
in-house replacement for that engine's model executor.
"""
from __future__ import annotations

import logging
import math
import os
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

from ..config import ModelConfig
from ..ops import gemm, pgemm
from ..ops import quant as Q
from ..ops import reference as ref
from ..parallel.comm import TPGroup

log = logging.getLogger(__name__)

DG_MOE_STEPS = (1, 2, 3, 4, 6, 7, 8, 16)  # 256-k steps per K slice the expert decode GEMM is built for
MOE_KERNEL_MAX_PAIRS = 2048  # larger (prefill) batches use per-expert hipBLASLt GEMMs ...
MOE_KERNEL_MAX_ROWS_PER_EXPERT = 1024  # ... unless the experts are many and small (Qwen3-MoE: 128 x 768)


@dataclass
class AttnMeta:
    """Per-step attention metadata (prefill rows first, then decode rows)."""
    num_prefill_tokens: int
    num_decode: int
    positions: torch.Tensor            # long [T]
    slot_mapping: torch.Tensor         # long [T]
    # prefill
    bt_prefill: torch.Tensor | None = None   # int32 [np, max_blocks]
    cu_q: torch.Tensor | None = None         # int32 [np+1]
    ctx_prefill: torch.Tensor | None = None  # int32 [np]
    tiles: torch.Tensor | None = None        # int32 [nt, 2]
    # decode
    bt_decode: torch.Tensor | None = None    # int32 [nd, max_blocks]
    ctx_decode: torch.Tensor | None = None   # int32 [nd]
    tmp_out: torch.Tensor | None = None
    tmp_ml: torch.Tensor | None = None
    # multimodal prefill (Qwen3-VL): per-row rotary table (positions = row index),
    # image embeddings for rows mm_rows and DeepStack features added after layers 0..n-1
    cos_sin: torch.Tensor | None = None
    mm_rows: torch.Tensor | None = None
    mm_embeds: torch.Tensor | None = None
    mm_deepstack: list | None = None
    # decode lookahead (model_runner): (src, tok) — row i's input id is tok[src[i]]
    # where src[i] >= 0 (the previous graph step's sampled id), else ids[i]
    id_src: tuple | None = None


@dataclass
class LayerWeights:
    ln1: torch.Tensor
    wqkv: torch.Tensor
    wo: torch.Tensor
    ln2: torch.Tensor
    # dense MLP
    wgu: torch.Tensor | None = None
    wd: torch.Tensor | None = None
    # MoE
    router: torch.Tensor | None = None       # [E, H]
    w13: torch.Tensor | None = None          # [E, 2*I/TP, H]
    w2: torch.Tensor | None = None           # [E, H, I/TP]
    moe_packed: tuple | None = None          # (w13 gate/up-interleaved, w2) packed per expert for decode
    quant: dict = field(default_factory=dict)  # GGUF-quantized GEMM weights by name
    # family extras (Qwen2 bias, Qwen3/Gemma-3 per-head q/k norms, Gemma-3 sandwich norms)
    bqkv: torch.Tensor | None = None         # [(nq + 2 nkv) * D / TP]
    q_norm: torch.Tensor | None = None       # [D] fp32
    k_norm: torch.Tensor | None = None       # [D] fp32
    post_attn_norm: torch.Tensor | None = None
    post_ff_norm: torch.Tensor | None = None


def shard_sizes(cfg: ModelConfig, tp: int):
    assert cfg.num_heads % tp == 0, f"num_heads {cfg.num_heads} not divisible by TP {tp}"
    nq = cfg.num_heads // tp
    if cfg.num_kv_heads >= tp:
        assert cfg.num_kv_heads % tp == 0
        nkv = cfg.num_kv_heads // tp
    else:
        assert tp % cfg.num_kv_heads == 0
        nkv = 1  # kv heads replicated across ranks
    I = cfg.expert_size if cfg.num_experts else cfg.intermediate_size
    assert I % tp == 0
    inter = I // tp
    vpad = (cfg.vocab_size + tp - 1) // tp
    return nq, nkv, inter, vpad


class LlamaModel:
    # load FP8 checkpoints natively (e4m3 + scales, ops/quant.py) instead of
    # dequantising them to bf16 at load (weights/safetensors_loader.py)
    native_fp8 = True
    # fused decode: qkv partials -> RoPE + KV write + attention in one kernel
    # (attention_decode.hip QkvIn), opt-in with HIPSERVE_FUSED_QKV_ATTN=1. Bit-exact.
    # First version: 5.57 vs 5.49 ms per Llama-3-8B B=64 decode step (every wave re-read
    # the fp32 partials for q before streaming K/V). Now each wave's first K/V chunk is
    # issued before the partial sums and q is computed once per workgroup (shared via
    # LDS): 5.322 / 5.332 vs 5.332 / 5.327 ms in round 2 (parity). Re-measured in round 6
    # after the non-temporal K/V stream and DPP reductions: 5.257 / 5.247 vs 5.306 / 5.297 ms
    # (tools/decode_gap.py, alternating runs, profiles/r6_fused_qkv_attn_ab.log) — now the
    # default for bf16 caches without q/k norm, qkv bias or sliding window; =0 restores the
    # separate splitk_rope_cache launch
    fused_qkv_attention = os.environ.get("HIPSERVE_FUSED_QKV_ATTN", "1") == "1"
    # (round 3 tried a "v2" decode layer with the split-K fix-up and the epilogue inside each
    # decode GEMM launch: slower, 6,398 vs 7,650 tok/s, profiles/r3_bench_v2_first.json —
    # an in-launch split-K seam costs more than the kernel boundary it replaces; removed)

    def __init__(self, cfg: ModelConfig, tp: TPGroup, device, dtype=torch.bfloat16, ops=None,
                 max_pos: int | None = None):
        self.cfg = cfg
        self.tp = tp
        self.device = torch.device(device)
        self.dtype = dtype
        self.kv_dtype = dtype  # paged KV cache element (ModelRunner: float8_e4m3fn for --kv-cache-dtype fp8)
        self.ops = ops
        self.nq, self.nkv, self.inter, self.vpad = shard_sizes(cfg, tp.world_size)
        self.D = cfg.head_dim
        self.scale = cfg.attn_scale or 1.0 / math.sqrt(self.D)
        self.layers: list[LayerWeights] = []
        self.embed: torch.Tensor | None = None
        self.norm: torch.Tensor | None = None
        self.lm_head: torch.Tensor | None = None
        mp = max_pos or cfg.max_position_embeddings
        self.cos_sin = ref.rope_cos_sin(self.D, mp, cfg.rope_theta, cfg.rope_scaling).to(self.device)
        # sliding-window layers with their own RoPE base (Gemma-3 local layers: plain RoPE)
        self.cos_sin_local = self.cos_sin
        if cfg.rope_local_theta and any(cfg.layer_windows):
            self.cos_sin_local = ref.rope_cos_sin(self.D, mp, cfg.rope_local_theta, None).to(self.device)
        self.vanilla = not (cfg.qkv_bias or cfg.qk_norm or cfg.sandwich_norm or cfg.hidden_act != "silu"
                            or any(cfg.layer_windows) or cfg.embed_scale != 1.0)
        # families the fused decode layer covers: Llama-style plus q/k/v bias (Qwen2),
        # per-head q/k RMSNorm (Qwen3; folded into the split-K RoPE epilogue), MoE MLPs
        # (Mixtral, Qwen3-MoE / Qwen3-VL-MoE) and Gemma-3 (sandwich norms in
        # splitk_post_add_rmsnorm at TP = 1, reduce + all-reduce + norms at TP > 1;
        # GeGLU over the gate|up partials, sliding-window
        # layers with their local RoPE table, embedding scale)
        self.fused_family = (cfg.hidden_act in ("silu", "gelu_tanh")
                             and (not cfg.qk_norm or (cfg.rope_mode == 0 and self.D in (64, 128, 256))))
        self.decode_partition = 512
        self.block_size_hint = 16  # KV block size (set by the runner)
        self.quant_linear = None  # set by the GGUF loader: callable(x, qweight) -> y
        self.fused_decode = True  # decode-only batches: split-K partials -> fused epilogues
        self.visual = None        # models.vision.VisionTower (Qwen3-VL), replicated on every TP rank
        if cfg.vision is not None:
            from .vision import VisionTower

            self.visual = VisionTower(cfg.vision, self.device, dtype, ops)

    # ---------------------------------------------------------------- weights
    def allocate_random(self, seed: int = 0, std: float = 0.02):
        """Synthetic weights generated on the device (K16, csrc/kernels/init.hip):
        uniform with standard deviation ``std``, keyed by each element's position in
        the UNSHARDED tensor, so every TP rank holds exactly its shard of the same
        model and dummy weights are identical for any TP degree."""
        cfg, dev, dt = self.cfg, self.device, self.dtype
        H, D = cfg.hidden_size, self.D
        rank, tp = self.tp.rank, self.tp.world_size
        scale = std * math.sqrt(3.0)
        names = {}

        def fill(view, key, row0, col0, gcols):
            k = (seed * 1000003 + names.setdefault(key, len(names) + 1) * 7919) & 0xFFFFFFFF
            self.ops.fill_uniform(view, row0, col0, gcols, k, scale)

        def new(*shape):
            return torch.empty(*shape, device=dev, dtype=dt)

        nd = torch.float32 if cfg.norm_offset else dt  # Gemma norms are fp32 (1 + w)

        def ones(n, dtype=None):
            return torch.ones(n, device=dev, dtype=dtype or nd)

        self.embed = new(self.vpad, H)
        fill(self.embed, "embed", rank * self.vpad, 0, H)
        self.norm = ones(H)
        if cfg.tie_word_embeddings:
            self.lm_head = self.embed
        else:
            self.lm_head = new(self.vpad, H)
            fill(self.lm_head, "lm_head", rank * self.vpad, 0, H)
        nq, nkv, I = self.nq, self.nkv, self.inter
        kv_head0 = rank * nkv if cfg.num_kv_heads >= tp else rank // (tp // cfg.num_kv_heads)
        self.layers = []
        for li in range(cfg.num_layers):
            lw = LayerWeights(ln1=ones(H), wqkv=new((nq + 2 * nkv) * D, H), wo=new(H, nq * D), ln2=ones(H))
            fill(lw.wqkv[:nq * D], f"{li}.q", rank * nq * D, 0, H)
            fill(lw.wqkv[nq * D:(nq + nkv) * D], f"{li}.k", kv_head0 * D, 0, H)
            fill(lw.wqkv[(nq + nkv) * D:], f"{li}.v", kv_head0 * D, 0, H)
            fill(lw.wo, f"{li}.o", 0, rank * nq * D, cfg.num_heads * D)
            if cfg.qkv_bias:
                lw.bqkv = torch.zeros((nq + 2 * nkv) * D, device=dev, dtype=dt)
            if cfg.qk_norm:
                lw.q_norm, lw.k_norm = ones(D, torch.float32), ones(D, torch.float32)
            if cfg.sandwich_norm:
                lw.post_attn_norm, lw.post_ff_norm = ones(H), ones(H)
            if cfg.num_experts:
                E, Ig = cfg.num_experts, cfg.expert_size
                lw.router = new(E, H)
                fill(lw.router, f"{li}.router", 0, 0, H)
                lw.w13 = new(E, 2 * I, H)
                lw.w2 = new(E, H, I)
                for e in range(E):
                    fill(lw.w13[e, :I], f"{li}.w1", e * Ig + rank * I, 0, H)
                    fill(lw.w13[e, I:], f"{li}.w3", e * Ig + rank * I, 0, H)
                    fill(lw.w2[e], f"{li}.w2", e * H, rank * I, Ig)
            else:
                lw.wgu = new(2 * I, H)
                fill(lw.wgu[:I], f"{li}.gate", rank * I, 0, H)
                fill(lw.wgu[I:], f"{li}.up", rank * I, 0, H)
                lw.wd = new(H, I)
                fill(lw.wd, f"{li}.down", 0, rank * I, cfg.intermediate_size)
            self.layers.append(lw)
        if self.visual is not None:
            self.visual.allocate_random(seed)

    # synthetic GGUF schemes (GGUF-tier benchmarks): per projection ggml type;
    # q4_k_m mirrors llama.cpp's Q4_K_M mix (attn_v, ffn_down, output in Q6_K)
    QUANT_SCHEMES = {
        "q4_k_m": {"q": 12, "k": 12, "v": 14, "o": 12, "gate": 12, "up": 12, "down": 14, "output": 14},
        "q8_0": {n: 8 for n in ("q", "k", "v", "o", "gate", "up", "down", "output")},
        "q4_0": {**{n: 2 for n in ("q", "k", "v", "o", "gate", "up", "down")}, "output": 14},
    }

    def allocate_random_quant(self, scheme: str, seed: int = 0):
        """Random-init model with GGUF-quantised projections (``QuantWeight``, the
        fused dequant-GEMM kernels of csrc/kernels/gguf.hip): random valid ggml
        blocks of each projection's format. Off the GPU the same blocks are
        dequantised to dense weights (CPU plumbing / numerics oracle)."""
        import numpy as np

        from ..ops import quant as Q
        from ..weights import gguf as G

        if scheme.lower() in ("fp8", "int8"):
            return self.allocate_random_fp8(seed, scheme.lower())
        if self.tp.world_size != 1:
            raise NotImplementedError("the GGUF tier runs TP=1 (one device per pod, like llama-server)")
        types = self.QUANT_SCHEMES[scheme.lower()]
        cfg, dev, dt = self.cfg, self.device, self.dtype
        H, D, I = cfg.hidden_size, self.D, cfg.intermediate_size
        nq, nkv, V = cfg.num_heads, cfg.num_kv_heads, cfg.vocab_size
        rng = np.random.default_rng(seed)

        def qtype(kind, k):  # llama.cpp-style fallback when K is not a multiple of the super-block
            t = types[kind]
            return t if k % G.BLOCK[t][0] == 0 else G.Q8_0

        def mat(*specs):  # (kind, N, K) parts stacked along N
            raws = [(qtype(k, kk), n, kk, Q.random_blocks(rng, qtype(k, kk), n, kk)) for k, n, kk in specs]
            if dev.type == "cuda":
                return Q.QuantWeight.from_raw(raws, dev)
            return torch.cat([torch.from_numpy(G.dequantize(r, t, n * kk).reshape(n, kk)).to(dt)
                              for t, n, kk, r in raws], 0)

        g = torch.Generator().manual_seed(seed)
        self.embed = (torch.randn(V, H, generator=g) * 0.02).to(device=dev, dtype=dt)
        self.norm = torch.ones(H, device=dev, dtype=dt)
        self.lm_head = mat(("output", V, H))
        self.layers = []
        for _ in range(cfg.num_layers):
            self.layers.append(LayerWeights(
                ln1=torch.ones(H, device=dev, dtype=dt),
                wqkv=mat(("q", nq * D, H), ("k", nkv * D, H), ("v", nkv * D, H)),
                wo=mat(("o", H, nq * D)), ln2=torch.ones(H, device=dev, dtype=dt),
                wgu=mat(("gate", I, H), ("up", I, H)), wd=mat(("down", H, I))))
        self.quant_linear = Q.quant_linear

    def allocate_random_fp8(self, seed: int = 0, kind: str = "fp8"):
        """Random-init model whose projections are 8-bit weights with per-output-channel
        scales, kept native in HBM (ops/quant.py): ``fp8`` = e4m3 (the layout of the
        reference's "FP8-Dynamic" checkpoints), ``int8`` = symmetric int8 weight-only
        (the reference's AWQ-8bit export). MoE experts become ``QuantMoE`` stacks for
        the quantised expert GEMM. Embeddings, norms, router and lm_head stay bf16 (the
        checkpoints' ``ignore`` list). Off the GPU the same 8-bit values are
        dequantised to dense weights."""
        from ..ops import quant as Q

        self.allocate_random(seed=seed)  # norms, embeddings, lm_head, bf16 projections (replaced below)
        dev = self.device

        def q8(w, rowpar=False):  # -> (QuantPart or None, dequantised dense)
            # per-output-channel scale over the WHOLE row: a row-parallel shard (o / down /
            # expert w2 at TP > 1) takes the max over the ranks' K slices, so every TP
            # degree quantises the same model as TP = 1 (a sharded checkpoint's scale)
            wf = w.float()
            amax = wf.abs().amax(1, keepdim=True)
            if rowpar and self.tp.world_size > 1:
                amax = self.tp.max_(amax)
            if kind == "int8":
                s = amax.clamp_min(1e-12) / 127.0
                qi = torch.round(wf / s).clamp(-127, 127)
                dense = (qi * s).to(self.dtype)
                ok = dev.type == "cuda" and w.shape[0] % 16 == 0 and w.shape[1] % 256 == 0
                return (Q.QuantPart.from_int8((qi + 128).to(torch.uint8), s, None, dev) if ok else None), dense
            s = amax.clamp_min(1e-12) / 448.0
            q = (wf / s).to(torch.float8_e4m3fn)
            ok = dev.type == "cuda" and w.shape[0] % 16 == 0 and w.shape[1] % 256 == 0
            return (Q.QuantPart.from_fp8(q, s, dev) if ok else None), (q.float() * s).to(self.dtype)

        def quant(w, splits, rowpar=False):
            parts = [q8(t, rowpar) for t in torch.split(w, splits, 0)]
            if all(p is not None for p, _ in parts):
                return Q.QuantWeight([p for p, _ in parts])
            return torch.cat([d for _, d in parts])

        def experts(w, rowpar=False):
            parts = [q8(w[e], rowpar) for e in range(w.shape[0])]
            if all(p is not None for p, _ in parts) and Q.QuantMoE.supported(parts[0][0].kqt, *w.shape[1:]):
                return Q.QuantMoE([p for p, _ in parts], kmajor=not rowpar)  # w13: super-chunk major
            return torch.stack([d for _, d in parts])

        D = self.D
        for lw in self.layers:
            lw.wqkv = quant(lw.wqkv, [self.nq * D, self.nkv * D, self.nkv * D])
            lw.wo = quant(lw.wo, [lw.wo.shape[0]], rowpar=True)
            if lw.wgu is not None:
                lw.wgu = quant(lw.wgu, [self.inter, self.inter])
                lw.wd = quant(lw.wd, [lw.wd.shape[0]], rowpar=True)
            if lw.w13 is not None:
                lw.w13, lw.w2 = experts(lw.w13), experts(lw.w2, rowpar=True)
        if dev.type == "cuda":
            torch.cuda.empty_cache()
        self.quant_linear = Q.quant_linear

    def quant_moes(self) -> list:
        """Every quantised expert stack (QuantMoE)."""
        from ..ops import quant as Q
        return [w for lw in self.layers for w in (lw.w13, lw.w2) if isinstance(w, Q.QuantMoE)]

    # ---------------------------------------------------------------- forward
    def linear(self, x: torch.Tensor, w, name: str | None = None) -> torch.Tensor:
        if isinstance(w, (torch.Tensor, gemm.PackedLinear)):
            return gemm.linear(x, w)
        return self.quant_linear(x, w)

    def gemm_shapes(self):
        """(N, K) of every dense bf16 projection (for the decode GEMM autotune)."""
        out = set()
        for lw in self.layers[:1]:
            for w in (lw.wqkv, lw.wo, lw.wgu, lw.wd, lw.router):  # + the MoE router [E, H] (E % 16 == 0)
                if (isinstance(w, (torch.Tensor, gemm.PackedLinear)) and w.dim() == 2
                        and (w is not lw.router or w.shape[0] % 16 == 0)):
                    out.add(tuple(w.shape))
        if isinstance(self.lm_head, (torch.Tensor, gemm.PackedLinear)):
            out.add(tuple(self.lm_head.shape))
        return sorted(out)

    def pack_decode_weights(self, shapes) -> int:
        """Pre-shuffled copies (ops/gemm.py ``PACKED``) of the dense projections whose
        (N, K) the decode tuner assigned to the packed decode GEMM. Costs one extra
        copy of those weights in HBM (288 GB per MI355X: bandwidth over capacity).
        With the fused decode path the merged gate|up weight is packed
        gate/up-interleaved instead (``PACKED_GLU``: the SiLU-GLU runs in its epilogue)."""
        n = 0
        glu = self.fused_decode and self.fused_family and self.cfg.hidden_act == "silu"
        # HBM budget: a packed copy is only made while >= 24 GiB + a quarter of the
        # device stay free for the KV cache (a 70B model on ONE 288 GB MI355X keeps
        # most weights unpacked; the tuner's packed choice then runs on the plain layout)
        reserve = 24 << 30
        if self.device.type == "cuda":
            reserve += torch.cuda.get_device_properties(self.device).total_memory // 4

        def fits(w):
            if self.device.type != "cuda":
                return True
            free, _ = torch.cuda.mem_get_info(self.device)
            return free - w.numel() * w.element_size() >= reserve

        for lw in self.layers:
            for w in (lw.wqkv, lw.wo, lw.wgu, lw.wd, lw.router):
                if (isinstance(w, torch.Tensor) and w.dim() == 2 and tuple(w.shape) in shapes
                        and fits(w)):
                    gemm.register_packed(w, glu=glu and w is lw.wgu and w.shape[0] % 128 == 0)
                    n += w.numel() * w.element_size()
        w = self.lm_head
        if isinstance(w, torch.Tensor) and w.dim() == 2 and tuple(w.shape) in shapes and fits(w):
            gemm.register_packed(w)
            n += w.numel() * w.element_size()
        return n + self.pack_moe_weights()

    def single_layout_ok(self) -> bool:
        """Families whose dense projections can live ONLY in the packed layout
        (``gemm.PackedLinear``): the fused decode path and the packed prefill GEMM cover
        every use — bf16 weights, SiLU-GLU (or MoE) MLPs, HIP ops, no exact-fp32 TP
        reduction (whose prefill GEMMs write fp32)."""
        return (getattr(self.ops, "name", "") == "hip" and self.fused_decode and self.fused_family
                and self.cfg.hidden_act == "silu" and not self.tp.exact_reduce and self.dtype == torch.bfloat16
                and hasattr(torch.ops.hipserve, "prefill_gemm_packed"))

    def to_single_layout(self) -> tuple[int, int]:
        """Replace every dense projection (qkv, o, gate|up, down, an untied lm_head) by its
        packed copy (``gemm.PackedLinear``; gate|up GLU-interleaved) and drop the
        row-major original: ONE resident copy per weight. One
        weight at a time, so the peak is the model plus one projection. Returns (weights
        converted, bytes freed)."""
        n = freed = 0

        def conv(w, glu=False):
            nonlocal n, freed
            if not (isinstance(w, torch.Tensor) and w.dim() == 2 and w.dtype == torch.bfloat16
                    and gemm.packable(*w.shape) and (not glu or w.shape[0] % 128 == 0)):
                return w
            wp = (gemm.glu_of(w) if glu else gemm.packed_of(w))
            if wp is None:
                wp = gemm.pack(w, glu=glu)
            # the registries are keyed by the plain tensor, which goes away now (other
            # engines in this process keep their entries)
            gemm.PACKED.pop(w.data_ptr(), None)
            gemm.PACKED_GLU.pop(w.data_ptr(), None)
            n += 1
            freed += w.numel() * w.element_size()
            return gemm.PackedLinear(wp, w.shape[0], w.shape[1], glu=glu)

        for lw in self.layers:
            lw.wqkv = conv(lw.wqkv)
            lw.wo = conv(lw.wo)
            if lw.wgu is not None:
                lw.wgu = conv(lw.wgu, glu=True)
                lw.wd = conv(lw.wd)
        if self.lm_head is not self.embed:
            self.lm_head = conv(self.lm_head)
        # MoE experts: their packed decode copy serves prefill too (the packed grouped
        # GEMM), so the row-major experts go, layer by layer
        freed += self.pack_moe_weights(drop_plain=True)
        if self.device.type == "cuda":
            torch.cuda.empty_cache()
        return n, freed

    def pack_moe_weights(self, drop_plain: bool = False) -> int:
        """Per-expert packed copies of the MoE weights for the decode expert GEMM
        (``moe_hip``): w13 gate/up-interleaved (SiLU-GLU in the GEMM epilogue), w2
        plain. The row-major originals stay for prefill (per-expert hipBLASLt), so
        this doubles the expert bytes (Mixtral-8x7B: +90 GB of 288 GB) — skipped
        when less than 24 GiB of HBM would stay free for the KV cache, or with
        HIPSERVE_MOE_PACK=0 (the row-major expert GEMM runs instead)."""
        if (not self.cfg.num_experts or getattr(self.ops, "name", "") != "hip"
                or os.environ.get("HIPSERVE_MOE_PACK", "1") == "0"):
            return 0
        lws = [lw for lw in self.layers if isinstance(lw.w13, torch.Tensor) and self._moe_decode_ok(lw)]
        if not lws:
            return 0
        need = sum(2 * (lw.w13.numel() + lw.w2.numel()) for lw in lws)
        if drop_plain:  # the packed copy REPLACES the row-major experts (one layer at a time)
            if not all(lw.moe_packed is not None or self.cfg.hidden_act == "silu" for lw in lws):
                return 0
            need = 0
        if self.device.type == "cuda":
            free, _ = torch.cuda.mem_get_info(self.device)
            if need + (24 << 30) > free:
                log.warning("MoE decode weights not packed: %.1f GB needed, %.1f GB free", need / 2**30, free / 2**30)
                return 0
        op = torch.ops.hipserve
        freed = 0
        for lw in lws:
            if lw.moe_packed is None:
                E, N13, K13 = lw.w13.shape
                _, N2, K2 = lw.w2.shape
                p13 = torch.empty(E, N13 * K13, dtype=lw.w13.dtype, device=lw.w13.device)
                p2 = torch.empty(E, -(-N2 // 128) * 128 * K2, dtype=lw.w2.dtype, device=lw.w2.device)
                op.pack_decode_weight(p13, lw.w13.contiguous(), True)  # all experts in one launch
                op.pack_decode_weight(p2, lw.w2.contiguous(), False)
                lw.moe_packed = (p13, p2)
            if drop_plain and self.moe_packed_prefill(lw, for_drop=True):
                freed += 2 * (lw.w13.numel() + lw.w2.numel())
                lw.w13 = lw.w2 = None
        return freed if drop_plain else need

    def fused_gemm_shapes(self) -> dict:
        """{(N, K): epilogue spec} of the projections whose decode GEMM output feeds
        a fused epilogue (ops/gemm.py tunes them as GEMM + epilogue units)."""
        if not self.layers or not self.fused_family:
            return {}
        lw = self.layers[0]
        out = {}
        dense = (torch.Tensor, gemm.PackedLinear)
        if isinstance(lw.wo, dense):
            out[tuple(lw.wo.shape)] = ("norm",)
        if isinstance(lw.wd, dense):
            out[tuple(lw.wd.shape)] = ("norm",)
        if isinstance(lw.wqkv, dense):
            # the fused decode attention consumes the partials itself (no epilogue launch):
            # timed as the partial GEMM alone; else GEMM + splitk_rope_cache
            kind = "attn" if self.fused_qkv_attn_ok() else "rope"
            out[tuple(lw.wqkv.shape)] = (kind, self.nq, self.nkv, self.D, self.cfg.rope_mode)
        if isinstance(lw.wgu, dense) and lw.wgu.shape[0] % 128 == 0 and self.cfg.hidden_act == "silu":
            out[tuple(lw.wgu.shape)] = ("glu",)  # GeGLU: plain partials + splitk_glu (tuned as a plain GEMM)
        return out

    def fused_qkv_attn_ok(self, layer: int | None = None) -> bool:
        """Decode attention straight from the qkv split-K partials (RoPE + KV write inside,
        attention_decode.hip QkvIn): bf16 cache, head_dim 64 / 128, no qkv bias, per-head q/k
        RMSNorm (Qwen3) only with rotate-half RoPE, no sliding window (``layer`` None: on
        every layer)."""
        lw0 = self.layers[0] if self.layers else None
        if (not self.fused_qkv_attention or self.D not in (64, 128) or lw0 is None or lw0.bqkv is not None
                or (lw0.q_norm is not None and self.cfg.rope_mode != 0)
                or torch.finfo(self.kv_dtype).bits != 16):
            return False
        layers = range(len(self.layers)) if layer is None else (layer,)
        return not any(self.cfg.window_of(i) for i in layers)

    def _fused_ok(self, meta: AttnMeta) -> bool:
        return (self.fused_decode and meta.num_prefill_tokens == 0
                and getattr(self.ops, "name", "") == "hip" and self.fused_family)

    def fused_embed_ok(self, meta: AttnMeta) -> bool:
        """The fused decode forward can take the lookahead ids unresolved (``meta.id_src``):
        id select + embedding gather + residual copy + first RMSNorm in one kernel
        (``embed_rmsnorm``, norm.hip), Gemma's embedding scale included. TP=1 only (the
        vocab-parallel embedding needs a cross-rank sum before the norm)."""
        return (self._fused_ok(meta) and self.tp.world_size == 1 and self.embed.dtype == torch.bfloat16
                and hasattr(torch.ops.hipserve, "embed_rmsnorm"))

    @staticmethod
    def resolve_ids(ids: torch.Tensor, meta: AttnMeta) -> torch.Tensor:
        if meta.id_src is None:
            return ids
        src, tok = meta.id_src
        return torch.where(src >= 0, tok.index_select(0, src.clamp(min=0)), ids)

    def add_rmsnorm(self, out, residual, x, splits, w, out16=None, out8=None, out8p=None):
        """residual += x summed over the TP ranks; out = RMSNorm(residual) * w.
        ``x`` is this rank's partial output of a row-parallel projection: fp32
        split-K partials [S, M, N] of a decode GEMM, or the plain projection output
        (bf16; fp32 under exact TP reduction). TP=1 runs the single-GPU fused
        kernels; TP>1 the in-house cross-rank epilogue (parallel/comm.py)."""
        eps = self.cfg.rms_norm_eps
        if self.tp.world_size > 1:
            assert out16 is None and out8 is None and out8p is None, "out16 / out8 need TP = 1"
            return self.tp.add_rmsnorm(out, residual, x, splits, w, eps, ops=self.ops)
        if x.dtype == torch.float32 and residual.dtype != torch.float32:
            q8, s8 = out8 if out8 is not None else (None, None)
            torch.ops.hipserve.splitk_add_rmsnorm(out, residual, x, splits, w, eps, out16, q8, s8)
        else:  # out8p: the FP8 prefill GEMM's e4m3 input (the decode out8 needs the partial path)
            assert out16 is None and out8 is None, "out16 / out8 need the split-K partial path"
            self.ops.fused_add_rmsnorm(out, x, residual, w, eps, out8=out8p)
        return out

    def post_add_rmsnorm(self, out, residual, pt, x, w, w_post, w_next, out16=None, out8=None):
        """Sandwich-norm epilogue (Gemma-3): residual += RMSNorm(sum over the TP ranks
        of x @ w.T) * w_post; out = RMSNorm(residual) * w_next. At TP = 1 one kernel
        over the split-K partials ``pt`` when the decode GEMM wrote them (also writing
        ``out16``, the f16 pair-order copy for a quantised consumer; returns True);
        otherwise the chain of ``forward`` — partials reduced (bf16, or fp32 under
        exact TP reduction) or the projection itself, the cross-rank sum, then the two
        norms (bit-identical to ``forward`` at TP = 1; returns False: no out16)."""
        eps = self.cfg.rms_norm_eps
        tp1 = self.tp.world_size == 1
        if tp1 and pt is not None and w_post.dtype == w_next.dtype and residual.dtype == torch.bfloat16:
            q8, s8 = out8 if out8 is not None else (None, None)
            torch.ops.hipserve.splitk_post_add_rmsnorm(out, residual, pt[0], pt[1], w_post, w_next, eps, out16, q8, s8)
            return True
        if pt is not None and not tp1 and self.tp.exact_reduce:
            S, (M, N) = pt[1], residual.shape  # fp32: the cross-rank sum rounds once
            o = pt[0].reshape(-1)[:S * M * N].view(S, M, N).sum(0)
        elif pt is not None:
            o = torch.empty_like(residual)
            torch.ops.hipserve.splitk_reduce(o, pt[0], pt[1])
        else:
            o = self.linear_rowpar(x, w)
        if not tp1:
            o = self._tp_sum(o, residual)
        self.ops.rmsnorm(o, o, w_post, eps)
        self.ops.fused_add_rmsnorm(out, o, residual, w_next, eps)
        return False

    def linear_rowpar(self, x: torch.Tensor, w) -> torch.Tensor:
        """Row-parallel projection (o_proj / down_proj). Under exact TP reduction
        the GEMM writes fp32, so the cross-rank sum rounds once, like TP=1's GEMM."""
        if (self.tp.world_size > 1 and self.tp.exact_reduce and x.is_cuda and isinstance(w, torch.Tensor)):
            return torch.mm(x, w.t(), out_dtype=torch.float32)
        return self.linear(x, w)

    def _tp_sum(self, x: torch.Tensor, like: torch.Tensor) -> torch.Tensor:
        """Plain all-reduce of a row-parallel output (the sandwich-norm families,
        whose post-norm needs the full sum before the residual add)."""
        self.tp.all_reduce(x)
        return x if x.dtype == like.dtype else x.to(like.dtype)

    def embed_tokens(self, ids: torch.Tensor) -> torch.Tensor:
        if self.tp.world_size == 1:
            return F.embedding(ids, self.embed)
        start = self.tp.rank * self.vpad
        local = ids - start
        mask = (local >= 0) & (local < self.vpad)
        h = F.embedding(local.clamp(0, self.vpad - 1), self.embed)
        h = h * mask.unsqueeze(-1).to(h.dtype)
        return self.tp.all_reduce(h)

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        ops, cfg = self.ops, self.cfg
        T = ids.shape[0]
        H, D, nq, nkv = cfg.hidden_size, self.D, self.nq, self.nkv
        eps = cfg.rms_norm_eps
        Tp, Td = meta.num_prefill_tokens, meta.num_decode
        if self._fused_ok(meta):
            return self.forward_decode_fused(ids, meta, kv_caches)
        ids = self.resolve_ids(ids, meta)
        h = self.embed_tokens(ids)
        if cfg.embed_scale != 1.0:  # Gemma: embeddings * sqrt(hidden), the scale rounded to the dtype
            h = h * float(torch.tensor(cfg.embed_scale, dtype=h.dtype))
        ds = None
        if meta.mm_rows is not None:  # image placeholders take the vision tower's embeddings
            h.index_copy_(0, meta.mm_rows, meta.mm_embeds.to(h.dtype))
            ds = meta.mm_deepstack
        cos_sin = self.cos_sin if meta.cos_sin is None else meta.cos_sin
        residual = h.clone()
        xn = torch.empty_like(h)
        attn = torch.empty(T, nq * D, device=h.device, dtype=h.dtype)
        if Td:
            part, tmp_out, tmp_ml = self._decode_split(Td, meta)
        x8 = self._x8p(xn, self.layers[0].wqkv)  # FP8 models: the norm writes the e4m3 GEMM input too
        ops.rmsnorm(xn, h, self.layers[0].ln1, eps, out8=x8)
        L = len(self.layers)
        tp1 = self.tp.world_size == 1
        for i, lw in enumerate(self.layers):
            # prefill-sized batches: FP8 W8A8 (ops/pgemm.py), the packed-layout GEMM of a
            # single-layout model (gemm.linear dispatches PackedLinear), else hipBLASLt
            if x8 is not None:
                qkv = pgemm.f8_gemm(xn, lw.wqkv, 0, x8=x8)
            else:
                qkv = self.linear(xn, lw.wqkv)
            if lw.bqkv is not None:
                qkv += lw.bqkv
            if lw.q_norm is not None:  # per-head RMSNorm of q and k, before RoPE
                ops.qk_rmsnorm(qkv, lw.q_norm, lw.k_norm, nq, nkv, D, eps)
            kc, vc = kv_caches[i]
            win = cfg.window_of(i)
            ops.rope_cache(qkv, meta.positions, meta.slot_mapping, self.cos_sin_local if win else cos_sin,
                           kc, vc, nq, nkv, D, cfg.rope_mode)
            if Tp:
                ops.prefill_attention(attn[:Tp], qkv[:Tp], kc, vc, meta.bt_prefill, meta.cu_q,
                                      meta.ctx_prefill, meta.tiles, nq, nkv, self.scale, win)
            if Td:  # rows past Tp + Td: prefill padding (model_runner._pad_rows)
                ops.paged_decode(attn[Tp:Tp + Td], qkv[Tp:Tp + Td], kc, vc, meta.bt_decode, meta.ctx_decode,
                                 tmp_out, tmp_ml, nq, nkv, part, self.scale, win)
            x8 = self._x8p(xn, lw.wgu, glu=True)
            if tp1 and lw.post_attn_norm is None and isinstance(lw.wo, gemm.PackedLinear) and T > 64:
                gemm.packed_prefill(attn, lw.wo, 1, out=residual)  # residual += o_proj(attn), packed layout
                ops.rmsnorm(xn, residual, lw.ln2, eps, out8=x8)
            elif tp1 and lw.post_attn_norm is None and Q.qprefill_ok(lw.wo, T):
                Q.qprefill(attn, lw.wo, 1, out=residual)  # GGUF blocks, residual add in the epilogue
                ops.rmsnorm(xn, residual, lw.ln2, eps, out8=x8)
            else:
                o = self.linear_rowpar(attn, lw.wo)
                if lw.post_attn_norm is not None:  # Gemma sandwich norm (after the TP reduction)
                    o = self._tp_sum(o, xn)
                    ops.rmsnorm(o, o, lw.post_attn_norm, eps)
                    ops.fused_add_rmsnorm(xn, o, residual, lw.ln2, eps, out8=x8)
                else:
                    self.add_rmsnorm(xn, residual, o, 1, lw.ln2, out8p=x8)
            nxt = self.layers[i + 1].ln1 if i + 1 < L else self.norm
            x8n = self._x8p(xn, self.layers[i + 1].wqkv) if i + 1 < L else None  # next layer's qkv input
            if lw.router is not None:
                h = self.moe(xn, lw)
            else:
                gelu = cfg.hidden_act == "gelu_tanh"
                act = act8 = None
                if pgemm.f8_use(lw.wgu, T, glu=True):  # FP8 gate|up
                    if pgemm.f8_use(lw.wd, T):  # FP8 down too: act straight to e4m3 (glu_quant)
                        act8 = pgemm.f8_glu_q8(xn, lw.wgu, gelu, x8)
                    if act8 is None:  # GLU in the e4m3 GEMM's epilogue
                        act = pgemm.f8_gemm(xn, lw.wgu, 3 if gelu else 2, x8=x8)
                elif isinstance(lw.wgu, gemm.PackedLinear) and lw.wgu.glu:  # GLU in the packed GEMM's epilogue
                    act = gemm.packed_glu(xn, lw.wgu, gelu)
                elif cfg.hidden_act in ("silu", "gelu_tanh") and Q.qprefill_ok(lw.wgu, T, glu=True):
                    act = Q.qprefill(xn, lw.wgu, 3 if gelu else 2)  # GGUF blocks, GLU in the epilogue
                if act8 is not None:
                    h = pgemm.f8_gemm(None, lw.wd, 0, x8=act8)
                elif act is None:
                    gu = self.linear(xn, lw.wgu)
                    act = torch.empty(T, self.inter, device=xn.device, dtype=xn.dtype)
                    self.act_and_mul(act, gu)
                if act8 is None and (tp1 and lw.post_ff_norm is None and not (ds is not None and i < len(ds))
                                     and (Q.qprefill_ok(lw.wd, T)
                                          or (isinstance(lw.wd, gemm.PackedLinear) and T > 64))):
                    if isinstance(lw.wd, gemm.PackedLinear):
                        gemm.packed_prefill(act, lw.wd, 1, out=residual)
                    else:
                        Q.qprefill(act, lw.wd, 1, out=residual)
                    ops.rmsnorm(xn, residual, nxt, eps, out8=x8n)
                    x8 = x8n
                    continue
                if act8 is None:
                    h = self.linear_rowpar(act, lw.wd)
            if ds is not None and i < len(ds) and self.tp.rank == 0:
                # DeepStack: visual features join the residual stream after layer i
                # (rank 0 only: the row-parallel partials are summed across ranks next)
                h = h.index_add(0, meta.mm_rows, ds[i].to(h.dtype))
            if lw.post_ff_norm is not None:
                h = self._tp_sum(h, xn)
                ops.rmsnorm(h, h, lw.post_ff_norm, eps)
                ops.fused_add_rmsnorm(xn, h, residual, nxt, eps, out8=x8n)
            else:
                self.add_rmsnorm(xn, residual, h, 1, nxt, out8p=x8n)
            x8 = x8n
        return xn

    def act_and_mul(self, out: torch.Tensor, gu: torch.Tensor):
        """GLU activation of the merged [gate | up] output: SiLU (Llama/Qwen/Mixtral)
        or tanh-GELU (Gemma GeGLU)."""
        if self.cfg.hidden_act == "gelu_tanh":
            return self.ops.gelu_and_mul(out, gu)
        return self.ops.silu_and_mul(out, gu)

    def forward_decode_fused(self, ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Decode-only forward with the decode GEMMs' split-K partials reduced
        inside the next op (at TP>1 the o_proj / down epilogues are the in-house
        cross-rank reduce + residual + RMSNorm kernel, ``add_rmsnorm``): qkv -> RoPE + KV write, o_proj -> residual add + RMSNorm,
        down -> residual add + the NEXT
        layer's RMSNorm (final norm after the last layer), SiLU-GLU in the gate|up
        GEMM's epilogue (gate/up-interleaved packing). Bit-identical to
        ``forward``; each fusion point falls back to the unfused op when the tuner
        picked hipBLASLt for that projection."""
        ops, cfg, op = self.ops, self.cfg, torch.ops.hipserve
        T = ids.shape[0]
        D, nq, nkv = self.D, self.nq, self.nkv
        eps = cfg.rms_norm_eps
        xn16 = None  # f16 pair-order copy of xn from its producer (quantised GEMM input)
        xn8 = None   # (e4m3 xn, row scales) from its producer (W8A8 FP8 decode GEMM input)
        if ids.dtype == torch.long and self.fused_embed_ok(meta):
            residual = torch.empty(T, cfg.hidden_size, device=ids.device, dtype=self.embed.dtype)
            xn = torch.empty_like(residual)
            xn8 = self._x8(xn, self.layers[0].wqkv)
            src, tok = meta.id_src if meta.id_src is not None else (None, None)
            # Gemma: embeddings * sqrt(hidden), the scale rounded to the dtype (as forward())
            scale = float(torch.tensor(cfg.embed_scale, dtype=self.embed.dtype))
            op.embed_rmsnorm(xn, residual, self.embed, ids, src, tok, self.layers[0].ln1, eps, scale,
                             *(xn8 if xn8 is not None else (None, None)))
            h = residual
        else:
            h = self.embed_tokens(self.resolve_ids(ids, meta))
            if cfg.embed_scale != 1.0:  # Gemma: as forward()
                h = h * float(torch.tensor(cfg.embed_scale, dtype=h.dtype))
            residual = h.clone()
            xn = torch.empty_like(h)
            ops.rmsnorm(xn, h, self.layers[0].ln1, eps)
        attn = torch.empty(T, nq * D, device=h.device, dtype=h.dtype)
        part, tmp_out, tmp_ml = self._decode_split(T, meta)
        # the fused qkv attention only with ONE context partition per (sequence, kv head):
        # with a split context every partition's workgroup re-sums the qkv partials, and
        # long contexts ran slower fused (Llama-3.1-8B 8K x 16: 1,189 vs 1,210 tok/s,
        # 32K x 4: 232 vs 239; profiles/r6_qkv_attn_long_ab.log)
        one_part = -(-meta.bt_decode.shape[1] * self.block_size_hint // part) == 1
        L = len(self.layers)
        lw0 = self.layers[0]
        for i, lw in enumerate(self.layers):
            kc, vc = kv_caches[i]
            win = cfg.window_of(i)
            # the fused kernel writes the new token's K / V as bf16 (an e4m3 cache takes
            # the separate splitk_rope_cache writer)
            fuse_qa = one_part and self.fused_qkv_attn_ok(i) and kc.element_size() == 2
            cs = self.cos_sin_local if win else self.cos_sin
            pt = self._partial(xn, lw.wqkv, xn16, xn8)
            attn16 = self._x16(attn, lw.wo)  # the attention's f16 pair-order copy for a quantised o_proj
            if pt is not None and fuse_qa:
                # RoPE + KV write + attention in one kernel, straight from the partials
                op.paged_decode_qkv(attn, pt[0], pt[1], meta.positions, meta.slot_mapping, self.cos_sin, kc, vc,
                                    meta.bt_decode, meta.ctx_decode, tmp_out, tmp_ml, nq, nkv, part, self.scale,
                                    0, cfg.rope_mode, attn16, lw.q_norm, lw.k_norm, eps)
            elif pt is not None:  # + q/k/v bias and per-head q/k RMSNorm of the family, if any
                ws, S = pt
                qkv = torch.empty(T, lw.wqkv.shape[0], device=h.device, dtype=h.dtype)
                op.splitk_rope_cache(qkv, ws, S, meta.positions, meta.slot_mapping, cs, kc, vc,
                                     nq, nkv, D, cfg.rope_mode, lw.bqkv, lw.q_norm, lw.k_norm, eps)
            else:
                qkv = self.linear(xn, lw.wqkv)
                if lw.bqkv is not None:
                    qkv += lw.bqkv
                if lw.q_norm is not None:
                    ops.qk_rmsnorm(qkv, lw.q_norm, lw.k_norm, nq, nkv, D, eps)
                ops.rope_cache(qkv, meta.positions, meta.slot_mapping, cs, kc, vc, nq, nkv, D,
                               cfg.rope_mode)
            if pt is None or not fuse_qa:
                ops.paged_decode(attn, qkv, kc, vc, meta.bt_decode, meta.ctx_decode, tmp_out, tmp_ml,
                                 nq, nkv, part, self.scale, win, attn16)
            pt = self._partial(attn, lw.wo, attn16)
            if lw.post_attn_norm is not None:  # Gemma sandwich norm
                xn16 = self._x16(xn, lw.wgu) if pt is not None else None
                xn8 = self._x8(xn, lw.wgu) if pt is not None else None
                if not self.post_add_rmsnorm(xn, residual, pt, attn, lw.wo, lw.post_attn_norm, lw.ln2, xn16, xn8):
                    xn16 = xn8 = None
            elif pt is not None:
                xn16 = self._x16(xn, lw.wgu) if lw.router is None else None
                xn8 = self._x8(xn, lw.wgu) if lw.router is None else None
                self.add_rmsnorm(xn, residual, pt[0], pt[1], lw.ln2, xn16, xn8)
            else:
                xn16 = xn8 = None
                self.add_rmsnorm(xn, residual, self.linear_rowpar(attn, lw.wo), 1, lw.ln2)
            nxt = self.layers[i + 1].ln1 if i + 1 < L else self.norm
            if lw.router is not None:  # MoE MLP: routed expert GEMMs, then residual + next norm
                # TP = 1: the expert combine adds the residual and runs the next norm itself
                # (moe_combine_add_rmsnorm, via _combine) and returns None
                self._moe_norm = ((xn, residual, nxt) if self.tp.world_size == 1 and self.ops.name == "hip"
                                  and residual.dtype == torch.bfloat16 else None)
                y = self.moe(xn, lw)
                self._moe_norm = None
                if y is not None:
                    self.add_rmsnorm(xn, residual, y, 1, nxt)
                continue
            gelu = cfg.hidden_act == "gelu_tanh"
            gc = None if gelu else gemm.glu_choice(T, lw.wgu)
            pt = (None if gc is not None or (isinstance(lw.wgu, torch.Tensor) and not gelu)
                  else self._partial(xn, lw.wgu, xn16, xn8))
            act16 = act8 = None
            if gc is not None:     # SiLU-GLU in the gate|up GEMM's epilogue
                act = gemm.gemm_glu(xn, lw.wgu, gc)
            elif pt is not None:   # quantised gate|up, or GeGLU: the GLU over the plain-layout partials
                act = torch.empty(T, self.inter, device=xn.device, dtype=xn.dtype)
                act16 = self._x16(act, lw.wd)
                op.splitk_glu(act, pt[0], pt[1], gelu, act16)
            elif isinstance(lw.wgu, gemm.PackedLinear) and lw.wgu.glu:
                # single weight layout: a GLU-interleaved gate|up has no plain x W^T (decode
                # graph buckets above 64 rows, GeGLU at any row count)
                act = gemm.packed_glu(xn, lw.wgu, gelu)
            else:
                gu = self.linear(xn, lw.wgu)
                act = torch.empty(T, self.inter, device=xn.device, dtype=xn.dtype)
                self.act_and_mul(act, gu)
            pt = self._partial(act, lw.wd, act16, act8)
            if lw.post_ff_norm is not None:
                xn16 = self._x16(xn, self.layers[i + 1].wqkv) if pt is not None and i + 1 < L else None
                xn8 = self._x8(xn, self.layers[i + 1].wqkv) if pt is not None and i + 1 < L else None
                if not self.post_add_rmsnorm(xn, residual, pt, act, lw.wd, lw.post_ff_norm, nxt, xn16, xn8):
                    xn16 = xn8 = None
            elif pt is not None:
                xn16 = self._x16(xn, self.layers[i + 1].wqkv) if i + 1 < L else None
                xn8 = self._x8(xn, self.layers[i + 1].wqkv) if i + 1 < L else None
                self.add_rmsnorm(xn, residual, pt[0], pt[1], nxt, xn16, xn8)
            else:
                xn16 = xn8 = None
                self.add_rmsnorm(xn, residual, self.linear_rowpar(act, lw.wd), 1, nxt)
        return xn

    def quant_weights(self) -> list:
        """Every GGUF-quantised projection (QuantWeight), lm_head included."""
        from ..ops import quant as Q
        ws = [self.lm_head] + [getattr(lw, n) for lw in self.layers for n in ("wqkv", "wo", "wgu", "wd")]
        return [w for w in ws if isinstance(w, Q.QuantWeight)]

    def _route(self, x: torch.Tensor, lw, k: int):
        """(weights [T, k] fp32, expert ids [T, k] int32) of the top-k softmax over the
        router logits x @ router^T. When the start-up timing picked the decode GEMM for the
        router at this row count, its fp32 split-K partials go straight into the top-k
        kernel, which sums and rounds them as splitk_reduce would (bit-identical, one
        launch fewer per MoE layer)."""
        op = torch.ops.hipserve
        T, dev = x.shape[0], x.device
        w = torch.empty(T, k, dtype=torch.float32, device=dev)
        ids = torch.empty(T, k, dtype=torch.int32, device=dev)
        fc = (gemm.fused_choice(T, lw.router)
              if x.is_cuda and x.stride(1) == 1 and x.stride(0) % 8 == 0 else None)
        if fc is not None:
            ws, S = gemm.gemm_partial(x, lw.router, fc)
            op.moe_topk_softmax(w, ids, ws, k, self.cfg.norm_topk_prob, S)
        else:
            op.moe_topk_softmax(w, ids, gemm.linear(x, lw.router), k, self.cfg.norm_topk_prob)
        return w, ids

    def _partial(self, x: torch.Tensor, w, x16: torch.Tensor | None = None, x8=None):
        """(fp32 split-K partials [S, M, N], S) of ``x @ w.T`` for a fused decode
        epilogue: the tuned bf16 decode GEMM, or the GGUF MFMA GEMM for a
        ``QuantWeight`` (``x16``: the producer's f16 copy of x, see ``_x16``); None
        when the projection runs unfused (hipBLASLt choice)."""
        if isinstance(w, (torch.Tensor, gemm.PackedLinear)):
            fc = gemm.fused_choice(x.shape[0], w)
            return gemm.gemm_partial(x, w, fc) if fc is not None else None
        from ..ops import quant as Q
        M = x.shape[0]
        # FP8 W8A8 above 64 rows: TP = 1 (the cross-rank epilogues are sized for <= 64 rows)
        if getattr(w, "v2", False) and x.is_cuda and (M <= Q.MAX_FUSED_M or (
                M <= Q.F8_DECODE_MAX_M and self.tp.world_size == 1 and Q.f8_decode_ok(w))):
            return Q.quant_partial(x, w, x16, x8)
        return None

    X16 = os.environ.get("HIPSERVE_QGEMM_X16", "1") != "0"
    # (a split-K GLU -> e4m3 act kernel, one block per row, measured slower than splitk_glu's
    # 700-block grid + act_quant on Gemma-3-27B FP8 — 2,794 / 2,806 vs 2,836 / 2,851 tok/s —
    # and was removed in round 4)

    def _x16(self, like: torch.Tensor, consumer):
        """f16 buffer for the pair-order copy of ``like`` that its producer
        (splitk_add_rmsnorm / splitk_glu / the decode attention) writes when the consumer is
        a quantised decode GEMM at 33-64 rows (gguf_mfma.hip stages it as is instead of
        converting x in every workgroup); None otherwise."""
        from ..ops import quant as Q
        if (not self.X16 or self.tp.world_size != 1 or not like.is_cuda or not 32 < like.shape[0] <= 64
                or not getattr(consumer, "v2", False) or not hasattr(torch.ops.hipserve, "splitk_glu")
                or Q.f8_decode_ok(consumer)):  # the W8A8 decode GEMM quantises x itself
            return None
        return torch.empty(like.shape, dtype=torch.float16, device=like.device)

    def _x8p(self, like: torch.Tensor, consumer, glu: bool = False):
        """(e4m3, row scales) buffers for the per-token FP8 copy of ``like`` that its
        producing RMSNorm writes when ``consumer`` runs the FP8 W8A8 prefill GEMM at this
        row count (= act_quant_fp8 of ``like``; one kernel and one pass over x fewer);
        None otherwise. TP = 1 (the TP > 1 norms are the cross-rank epilogue)."""
        if (self.tp.world_size != 1 or not like.is_cuda or isinstance(consumer, torch.Tensor)
                or getattr(self.ops, "name", "") != "hip" or not pgemm.f8_use(consumer, like.shape[0], glu)):
            return None
        return (torch.empty(like.shape, dtype=torch.uint8, device=like.device),
                torch.empty(like.shape[0], dtype=torch.float32, device=like.device))

    def _x8(self, like: torch.Tensor, consumer):
        """(e4m3 [M, K] uint8, row scales fp32 [M]) buffers for the per-token FP8 copy of
        ``like`` that its producer (splitk_add_rmsnorm / splitk_post_add_rmsnorm) writes
        when the consumer runs the W8A8 FP8 decode GEMM (bit-identical to quantising
        ``like`` afterwards; one act_quant_fp8 launch fewer); None otherwise."""
        from ..ops import quant as Q
        if (self.tp.world_size != 1 or not like.is_cuda or like.shape[0] > Q.F8_DECODE_MAX_M
                or not Q.f8_decode_ok(consumer)):
            return None
        return (torch.empty(like.shape, dtype=torch.uint8, device=like.device),
                torch.empty(like.shape[0], dtype=torch.float32, device=like.device))

    def _decode_split(self, Td: int, meta: AttnMeta):
        """Context partition size for the decode attention: with >= 512 (sequence,
        kv-head) workgroups the chip is full without splitting, so contexts up to
        2048 run as ONE partition (no partial-merge kernel; 6.3 vs 5.3 TB/s at
        B=64, ctx 1152, profiles/decode_partition_sweep.md); small batches split the
        context (512) to occupy the CUs. Workspace views are sized to the chosen
        partition count so the grid carries no dead partitions."""
        part = self.decode_partition
        width = meta.bt_decode.shape[1] * self.block_size_hint
        # one partition per (sequence, kv head) when the grid is already wide: from 512
        # workgroups at any width, from 128 when every context fits one 2048-token
        # partition (GQA 8:1 shapes such as Qwen3-30B-A3B: B = 64 x 4 kv heads, ctx 1152,
        # 29.0 vs 46.9 us; B = 32: 21.3 vs 29.4; at 64 workgroups splitting still wins,
        # 17.4 vs 19.1 — profiles/r5_decode_partition_sweep.log)
        if Td * self.nkv >= 512 or (Td * self.nkv >= 128 and width <= 2048):
            part = max(part, 2048)
        mp = max(1, -(-width // part))
        to, tm = meta.tmp_out, meta.tmp_ml
        if to is None or mp > to.shape[2]:
            return self.decode_partition, to, tm
        nq, D = to.shape[1], to.shape[3]
        to = to.view(-1)[: Td * nq * mp * D].view(Td, nq, mp, D)
        tm = tm.view(-1)[: Td * nq * mp * 2].view(Td, nq, mp, 2)
        return part, to, tm

    # (out, residual, norm weight) of the decode layer's MoE tail: set around ``moe`` by
    # forward_decode_fused at TP = 1 so the combine also does residual add + next RMSNorm
    _moe_norm: tuple | None = None

    def _combine(self, out: torch.Tensor, y: torch.Tensor, S: int, w, pair_slot, k: int):
        """Weighted combine of a token's k expert rows (bf16 ``y`` [slots, H] when S == 0,
        fp32 split-K partials [S, slots, H] else) into ``out``. Under ``_moe_norm`` the
        one-kernel combine + residual add + next-layer RMSNorm instead (bit-identical to
        combine then fused_add_rmsnorm): writes the norm output and the residual in place,
        returns None."""
        op = torch.ops.hipserve
        if self._moe_norm is not None:
            xn, residual, nw = self._moe_norm
            self._moe_norm = None
            op.moe_combine_add_rmsnorm(xn, residual, y, S, w, pair_slot, k, nw, self.cfg.rms_norm_eps)
            return None
        if S > 0:
            op.moe_combine_partial(out, y, w, pair_slot, k)
        else:
            op.moe_combine(out, y, w, pair_slot, k)
        return out

    def moe(self, x: torch.Tensor, lw: LayerWeights) -> torch.Tensor | None:
        """Sparse MoE: softmax over the E router logits, top-k experts, weights
        renormalised over the k (Mixtral; Qwen3-MoE when ``norm_topk_prob``).

        On the GPU every batch runs one of the two graph-capturable kernel paths:
        ``moe_hip`` (the weight-streaming expert decode GEMM; decode batches, and
        prefill batches below the start-up-timed crossover ``moe_packed_from_tokens``)
        or ``moe_grouped`` (the packed-layout one-launch grouped GEMM). The per-expert
        loop at the end is the CPU reference path only."""
        cfg = self.cfg
        k = cfg.num_experts_per_tok
        T = x.shape[0]
        P = T * k
        hip = self.ops.name == "hip"
        if lw.w13 is not None and not isinstance(lw.w13, torch.Tensor):  # quantised experts (ops/quant.py QuantMoE)
            if P <= MOE_KERNEL_MAX_PAIRS:
                return self.moe_quant(x, lw)
            from ..ops import quant as Q

            if (hip and self._moe_packed_shape_ok() and lw.w13.dense is None
                    and self.moe_prefill_choice(T) == "packed"):
                # experts dequantised straight into the packed layout, then the one-launch grouped GEMMs
                lw = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None, router=lw.router,
                                  moe_packed=(Q.moe_packed_scratch(lw.w13, 0, True),
                                              Q.moe_packed_scratch(lw.w2, 1, False)))
                return self.moe_grouped(x, lw)
            lw = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None, router=lw.router,
                              w13=Q.moe_dense(lw.w13, 0), w2=Q.moe_dense(lw.w2, 1))
        if hip:
            kernel_ok = (cfg.num_experts <= 128 and cfg.hidden_size % 256 == 0 and self.inter % 256 == 0
                         and (lw.w13 is not None or lw.moe_packed is not None))
            grouped_ok = self.moe_packed_prefill(lw)
            if kernel_ok and (P <= MOE_KERNEL_MAX_PAIRS or not grouped_ok
                              or (P <= MOE_KERNEL_MAX_ROWS_PER_EXPERT * cfg.num_experts
                                  and self.moe_prefill_choice(T) == "hip")):
                return self.moe_hip(x, lw)
            if grouped_ok:
                return self.moe_grouped(x, lw)
            raise NotImplementedError(f"MoE shape (E={cfg.num_experts}, H={cfg.hidden_size}, I={self.inter}) "
                                      "has no gfx950 expert kernel")
        logits = F.linear(x, lw.router).float()
        w, idx = torch.topk(torch.softmax(logits, dim=-1), k, dim=-1)
        if cfg.norm_topk_prob:
            w = w / w.sum(-1, keepdim=True)
        out = torch.zeros(T, cfg.hidden_size, device=x.device, dtype=torch.float32)
        flat_idx = idx.reshape(-1)
        flat_tok = torch.arange(T, device=x.device).repeat_interleave(k)
        flat_w = w.reshape(-1)
        order = torch.argsort(flat_idx)
        counts = torch.bincount(flat_idx, minlength=cfg.num_experts).tolist()
        start = 0
        for e, n in enumerate(counts):
            if n == 0:
                continue
            sel = order[start:start + n]
            start += n
            toks = flat_tok[sel]
            gu = F.linear(x[toks], lw.w13[e])
            act = torch.empty(n, self.inter, device=x.device, dtype=x.dtype)
            self.ops.silu_and_mul(act, gu)
            y = F.linear(act, lw.w2[e]).float() * flat_w[sel].unsqueeze(-1)
            out.index_add_(0, toks, y)
        return out.to(x.dtype)

    def _moe_decode_ok(self, lw: LayerWeights) -> bool:
        """Shapes the expert decode GEMM (decode_gemm.hip kMoe) takes: K = H for w13
        (one K slice of 256 * {1,2,4,7,8,16}) and K = I/TP for w2 (split over K)."""
        H, I = self.cfg.hidden_size, self.inter
        return ((H // 256) in DG_MOE_STEPS and H % 256 == 0 and I % 256 == 0 and (2 * I) % 128 == 0
                and self._moe_w2_splits(I, 1, 1) > 0)

    @staticmethod
    def _moe_w2_splits(K: int, ntiles: int, active: int) -> int:
        """Split-K factor of the w2 expert GEMM: the fewest K slices (of 256 * one of
        DG_MOE_STEPS) that give >= 1024 workgroups over the active expert tiles."""
        ks = K // 256
        opts = sorted(ks // st for st in DG_MOE_STEPS if ks % st == 0)
        if not opts:
            return 0
        for S in opts:
            if ntiles * S * active >= 1024:
                return S
        return opts[-1]

    def moe_grouped(self, x: torch.Tensor, lw: LayerWeights) -> torch.Tensor:
        """Prefill-sized MoE: routing (top-k kernel), expert-sorted slots padded to the
        GEMM's row tile (moe_align), then the two expert GEMMs as ONE launch each on the
        packed expert layout (prefill_gemm_packed.hip kGroup: expert ids read on the
        device, no host round trip, graph-capturable; the token rows gathered through the
        slot table inside the first GEMM's X loads, SiLU-GLU in its epilogue), and the
        weighted combine (moe_combine). Row-major experts without a packed copy (tests)
        are packed into a scratch first."""
        op = torch.ops.hipserve
        cfg = self.cfg
        E, k, H = cfg.num_experts, cfg.num_experts_per_tok, cfg.hidden_size
        T, dev = x.shape[0], x.device
        if lw.moe_packed is None:
            p13 = torch.empty(E, 2 * self.inter * H, dtype=lw.w13.dtype, device=dev)
            p2 = torch.empty(E, -(-H // 128) * 128 * self.inter, dtype=lw.w2.dtype, device=dev)
            op.pack_decode_weight(p13, lw.w13.contiguous(), True)
            op.pack_decode_weight(p2, lw.w2.contiguous(), False)
            lw = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None, router=lw.router, moe_packed=(p13, p2))
        P = T * k
        tile = 128 * gemm.PW_WM
        cap = -(-(P + E * (tile - 1)) // tile) * tile
        w, ids = self._route(x, lw, k)
        slots = torch.empty(cap, dtype=torch.int32, device=dev)
        tile_expert = torch.empty(cap // tile, dtype=torch.int32, device=dev)
        ntiles = torch.empty(1, dtype=torch.int32, device=dev)
        pair_slot = torch.empty(P, dtype=torch.int32, device=dev)
        ends = torch.empty(E, dtype=torch.int32, device=dev)
        op.moe_align(ids, E, tile, slots, tile_expert, ntiles, pair_slot, ends)
        p13, p2 = lw.moe_packed
        act = torch.empty(cap, self.inter, dtype=x.dtype, device=dev)
        # the first GEMM reads its token rows through the slot table (moe_gather fused)
        op.prefill_gemm_packed_grouped(act, x, p13, 2 * self.inter, 2, tile_expert, ntiles, gemm.PW_WM, gemm.PW_RW,
                                       slots, k)
        y = torch.empty(cap, H, dtype=x.dtype, device=dev)
        op.prefill_gemm_packed_grouped(y, act, p2, H, 0, tile_expert, ntiles, gemm.PW_WM, gemm.PW_RW)
        return self._combine(torch.empty(T, H, dtype=x.dtype, device=dev), y, 0, w, pair_slot, k)

    # prefill-sized MoE batches: the packed one-launch grouped GEMM (``moe_grouped``) or the
    # weight-streaming expert kernel (``moe_hip``). ``auto``: by the start-up timing of the
    # layer's expert shape at several token counts (``tune_moe_prefill``): the grouped GEMM
    # from ``moe_packed_from_tokens`` tokens up, the streaming kernel below (its 128-row
    # tiles are mostly padding when 128 experts share a few hundred tokens). ``1`` / ``0``
    # force the grouped GEMM / the streaming kernel. hipBLASLt's grouped GEMM
    # (torch._grouped_mm) lost to the packed kernel on every shipped MoE config (Mixtral
    # 4.82 vs 5.10 ms, Qwen3-30B-A3B 1.52 vs 5.17 ms per layer at 16K tokens,
    # profiles/r5_bench_mixtral_gather_fused.json, r5_bench_q3int8_align_multiblock.json)
    # and read its group offsets on the host: removed
    MOE_PACKED_PREFILL = os.environ.get("HIPSERVE_MOE_PACKED_PREFILL", "auto")
    moe_prefill_path: str | None = None  # "hip" | "packed" at the timed budget, set by tune_moe_prefill
    moe_packed_from_tokens: int = 0     # "packed": the grouped GEMM from this many tokens up

    @property
    def moe_prefill_packed(self) -> bool:
        return self.moe_prefill_path == "packed"

    def moe_prefill_choice(self, T: int) -> str:
        """'packed' (grouped GEMM) or 'hip' (streaming expert kernel) for a T-token batch."""
        mode = self.MOE_PACKED_PREFILL
        if mode in ("0", "1"):
            return "packed" if mode == "1" else "hip"
        if self.moe_prefill_path == "packed" and T >= self.moe_packed_from_tokens:
            return "packed"
        if self.moe_prefill_path is None:  # untimed (tests, CPU): the grouped GEMM above the kernel row limit
            E, k = self.cfg.num_experts, self.cfg.num_experts_per_tok
            return "packed" if T * k > MOE_KERNEL_MAX_ROWS_PER_EXPERT * E else "hip"
        return "hip"

    def _moe_packed_shape_ok(self) -> bool:
        return (self.cfg.hidden_act == "silu" and self.cfg.hidden_size % 256 == 0 and self.inter % 256 == 0
                and (2 * self.inter) % 128 == 0 and hasattr(torch.ops.hipserve, "prefill_gemm_packed_grouped"))

    def moe_packed_prefill(self, lw: LayerWeights, for_drop: bool = False) -> bool:
        """The packed-layout grouped GEMM can run this layer's prefill: SiLU-GLU experts,
        K of both GEMMs % 256, a packed copy (or row-major experts to pack from)."""
        if not self._moe_packed_shape_ok() or (lw.moe_packed is None and lw.w13 is None):
            return False
        if for_drop:
            return self.MOE_PACKED_PREFILL != "0" and lw.moe_packed is not None
        return True

    @torch.inference_mode()
    def tune_moe_prefill(self, T: int) -> dict | None:
        """Start-up timing of one MoE layer's prefill on random bf16 experts of the layer's
        shape through the model's own paths, the weight-streaming expert kernel
        (``moe_hip``, where its row limit allows) vs the packed one-launch grouped GEMM
        (``moe_grouped``), at ``T`` tokens and at halvings of it down to the decode
        kernels' pair limit. Sets ``moe_prefill_path`` (the winner at T) and
        ``moe_packed_from_tokens`` (the smallest timed count from which the grouped GEMM
        wins at every larger count). Cached per device and kernel build."""
        from ..ops import tune_cache as TC

        cfg = self.cfg
        lw = next((lw for lw in self.layers if lw.router is not None), None)
        if (lw is None or not self._moe_packed_shape_ok() or self.MOE_PACKED_PREFILL != "auto"
                or getattr(self.ops, "name", "") != "hip" or self.device.type != "cuda" or cfg.num_experts > 128):
            return None
        E, k, H, I = cfg.num_experts, cfg.num_experts_per_tok, cfg.hidden_size, self.inter
        quant = lw.w13 is not None and not isinstance(lw.w13, torch.Tensor)
        if not quant and lw.moe_packed is None and lw.w13 is None:
            return None
        key = [E, k, H, I, T, quant, "v2"]
        hit = TC.get(self.device, "moe_prefill", key)
        if hit is not None:
            self.moe_prefill_path, self.moe_packed_from_tokens = hit["path"], hit["packed_from_tokens"]
            return dict(hit, cached=True)
        op, dev = torch.ops.hipserve, self.device
        g = torch.Generator(device=dev).manual_seed(E * H + I)
        w13 = (torch.randn(E, 2 * I, H, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        w2 = (torch.randn(E, H, I, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        p13 = torch.empty(E, 2 * I * H, dtype=torch.bfloat16, device=dev)
        p2 = torch.empty(E, -(-H // 128) * 128 * I, dtype=torch.bfloat16, device=dev)
        op.pack_decode_weight(p13, w13, True)
        op.pack_decode_weight(p2, w2, False)
        router = (torch.randn(E, H, device=dev, generator=g) * 0.3).to(torch.bfloat16)
        syn = LayerWeights(ln1=None, wqkv=None, wo=None, ln2=None, router=router, w13=w13, w2=w2,
                           moe_packed=(p13, p2))
        counts = []
        t = T
        while t * k > MOE_KERNEL_MAX_PAIRS and len(counts) < 5:
            counts.append(t)
            t //= 2
        rows = []
        for t in counts:
            x = torch.randn(t, H, device=dev, generator=g).to(torch.bfloat16)
            # quantised experts dequantise once per step on either path: only the GEMMs are timed
            row = {"tokens": t, "packed_ms": round(pgemm._time(lambda i: self.moe_grouped(x, syn), reps=2), 3)}
            if not quant and t * k <= MOE_KERNEL_MAX_ROWS_PER_EXPERT * E and self._moe_decode_ok(syn):
                row["hip_ms"] = round(pgemm._time(lambda i: self.moe_hip(x, syn), reps=2), 3)
            rows.append(row)
        del w13, w2, p13, p2, syn
        torch.cuda.empty_cache()
        wins = [r.get("hip_ms") is None or r["packed_ms"] < r["hip_ms"] for r in rows]
        best = "packed" if not rows or wins[0] else "hip"
        frm = T
        for r, w_ in zip(rows, wins):  # counts descend: the grouped GEMM's run of wins from the top
            if not w_:
                break
            frm = r["tokens"]
        if best == "packed" and len(rows) and all(wins):
            frm = 0  # wins down to the pair limit: every prefill-sized batch
        self.moe_prefill_path, self.moe_packed_from_tokens = best, frm
        r = {"E": E, "H": H, "I": I, "tokens": T, "quant": quant, "path": best, "packed_from_tokens": frm,
             "timing": rows}
        TC.put(self.device, "moe_prefill", key, r)
        TC.flush()
        log.info("MoE prefill expert GEMMs: %s", r)
        return r

    def moe_hip(self, x: torch.Tensor, lw: LayerWeights) -> torch.Tensor:
        """Graph-capturable MoE on the gfx950 kernels (decode-sized batches): top-k
        routing, expert-sorted 16/32/64-row tiles, two gathered MFMA GEMMs with the
        SiLU*up in between, weighted combine. No host synchronisation.

        The expert GEMMs are the decode GEMM in its MoE mode (weight-streaming:
        128 weight rows x one expert tile per workgroup, x tile staged in LDS):
        with packed weights (``pack_moe_weights``) the SiLU-GLU runs in the w13
        epilogue, and w2 writes split-K fp32 partials that the combine sums."""
        op = torch.ops.hipserve
        cfg = self.cfg
        E, k, H = cfg.num_experts, cfg.num_experts_per_tok, cfg.hidden_size
        T, dev = x.shape[0], x.device
        P = T * k
        tile = 16 if P <= 8 * E else (32 if P <= 32 * E else 64)
        cap = -(-(P + E * (tile - 1)) // tile) * tile
        w, ids = self._route(x, lw, k)
        slots = torch.empty(cap, dtype=torch.int32, device=dev)
        tile_expert = torch.empty(cap // tile, dtype=torch.int32, device=dev)
        ntiles = torch.empty(1, dtype=torch.int32, device=dev)
        pair_slot = torch.empty(P, dtype=torch.int32, device=dev)
        op.moe_align(ids, E, tile, slots, tile_expert, ntiles, pair_slot)
        out = torch.empty(T, H, dtype=x.dtype, device=dev)
        if self._moe_decode_ok(lw):
            packed = lw.moe_packed is not None
            act = torch.empty(cap, self.inter, dtype=x.dtype, device=dev)
            if packed:
                op.moe_decode_gemm(act, x, lw.moe_packed[0], slots, tile_expert, tile, k, 2 * self.inter, 1,
                                   True, True)
            else:
                gu = torch.empty(cap, 2 * self.inter, dtype=x.dtype, device=dev)
                op.moe_decode_gemm(gu, x, lw.w13, slots, tile_expert, tile, k, 2 * self.inter, 1, False, False)
                self.ops.silu_and_mul(act, gu)
            active = min(E, cap // tile, P)
            S = self._moe_w2_splits(self.inter, -(-H // 128), active)
            w2 = lw.moe_packed[1] if packed else lw.w2
            if S == 1:  # one K slice: bf16 expert outputs, no fp32 partial slab
                y = torch.empty(cap, H, dtype=x.dtype, device=dev)
                op.moe_decode_gemm(y, act, w2, slots, tile_expert, tile, 0, H, 1, packed, False)
                return self._combine(out, y, 0, w, pair_slot, k)
            ws = torch.empty(S, cap, H, dtype=torch.float32, device=dev)
            op.moe_decode_gemm(ws, act, w2, slots, tile_expert, tile, 0, H, S, packed, False)
            return self._combine(out, ws, S, w, pair_slot, k)
        gu = torch.empty(cap, 2 * self.inter, dtype=x.dtype, device=dev)
        op.moe_gemm(gu, x, lw.w13, slots, tile_expert, tile, k)
        act = torch.empty(cap, self.inter, dtype=x.dtype, device=dev)
        self.ops.silu_and_mul(act, gu)
        y = torch.empty(cap, H, dtype=x.dtype, device=dev)
        op.moe_gemm(y, act, lw.w2, slots, tile_expert, tile, 0)
        return self._combine(out, y, 0, w, pair_slot, k)

    def moe_quant(self, x: torch.Tensor, lw: LayerWeights) -> torch.Tensor:
        """Decode-sized MoE on quantised experts (INT8 / FP8, ``QuantMoE``): routing and
        expert-sorted tiles as ``moe_hip``, then the dequant-MFMA expert GEMM in its
        MoE mode (gathered token rows, one expert's weight stream per workgroup) for
        w13, SiLU-GLU, and w2 (split over K into fp32 partials summed by the
        weighted combine). No host synchronisation (graph-capturable)."""
        op = torch.ops.hipserve
        cfg = self.cfg
        E, k, H = cfg.num_experts, cfg.num_experts_per_tok, cfg.hidden_size
        T, dev = x.shape[0], x.device
        P = T * k
        tile = 16 if P <= 8 * E else (32 if P <= 32 * E else 64)
        cap = -(-(P + E * (tile - 1)) // tile) * tile
        w, ids = self._route(x, lw, k)
        slots = torch.empty(cap, dtype=torch.int32, device=dev)
        tile_expert = torch.empty(cap // tile, dtype=torch.int32, device=dev)
        ntiles = torch.empty(1, dtype=torch.int32, device=dev)
        pair_slot = torch.empty(P, dtype=torch.int32, device=dev)
        op.moe_align(ids, E, tile, slots, tile_expert, ntiles, pair_slot)
        w13, w2 = lw.w13, lw.w2
        f32 = torch.empty(0, dtype=torch.float32, device=dev)
        act = torch.empty(cap, w13.N // 2, dtype=x.dtype, device=dev)
        if tile <= 32 and (w13.N // 2) % 16 == 0:  # GLU in the w13 epilogue (bit-identical)
            glu = 2 if cfg.hidden_act == "gelu_tanh" else 1
            op.qmoe_gemm(act, f32, x, w13.q, w13.rs, w13.kqt, w13.N, w13.K, slots, tile_expert, tile, k, 1,
                         w13.kmajor, glu)
        else:
            gu = torch.empty(cap, w13.N, dtype=x.dtype, device=dev)
            op.qmoe_gemm(gu, f32, x, w13.q, w13.rs, w13.kqt, w13.N, w13.K, slots, tile_expert, tile, k, 1,
                         w13.kmajor)
            self.act_and_mul(act, gu)
        out = torch.empty(T, H, dtype=x.dtype, device=dev)
        active = min(E, cap // tile, P)
        S = self._moe_w2_splits(w2.K, -(-H // 128), active)
        if S <= 1:
            y = torch.empty(cap, H, dtype=x.dtype, device=dev)
            op.qmoe_gemm(y, f32, act, w2.q, w2.rs, w2.kqt, w2.N, w2.K, slots, tile_expert, tile, 0, 1, w2.kmajor)
            return self._combine(out, y, 0, w, pair_slot, k)
        ws = torch.empty(S, cap, H, dtype=torch.float32, device=dev)
        S = op.qmoe_gemm(out, ws, act, w2.q, w2.rs, w2.kqt, w2.N, w2.K, slots, tile_expert, tile, 0, S, w2.kmajor)
        return self._combine(out, ws[:S], S, w, pair_slot, k)

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        logits = self.linear(hidden, self.lm_head)
        logits = self.tp.all_gather_lastdim(logits)
        return logits[:, : self.cfg.vocab_size]

    # ---------------------------------------------------------------- kv cache
    def kv_bytes_per_block(self, block_size: int) -> int:
        return 2 * self.cfg.num_layers * self.nkv * block_size * self.D * torch.finfo(self.kv_dtype).bits // 8

    def allocate_kv_cache(self, num_blocks: int, block_size: int):
        L = self.cfg.num_layers
        k = torch.zeros(L, num_blocks, self.nkv, block_size, self.D, device=self.device, dtype=self.kv_dtype)
        v = torch.zeros(L, num_blocks, self.nkv, self.D, block_size, device=self.device, dtype=self.kv_dtype)
        return [(k[i], v[i]) for i in range(L)]
