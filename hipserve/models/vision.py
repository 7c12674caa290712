"""Qwen3-VL vision tower on the hipserve op set (the reference's default HF model,
``Qwen3-VL-30B-A3B-Instruct-AWQ-8bit``: vllm-models/helm-chart/values.yaml:8-12,
served by vLLM with its vision encoder — here the encoder is in-house).

Pipeline per request (prefill only; the language model never sees pixels):

* patch embedding: the Conv3d of HF (kernel = stride = 2x16x16 over 3 channels) is a
  plain GEMM over the flattened 1536-value patches (hipBLASLt, bias in the epilogue);
* learned position table (48x48) resampled to each image's patch grid by bilinear
  interpolation with aligned corners — 4 gathered rows and weights per patch,
  computed on the host once per image;
* ``depth`` pre-LN ViT blocks: add+LayerNorm kernel -> qkv GEMM -> 2D RoPE (row
  angles on the first half of the rotary pairs, column angles on the second) +
  bidirectional attention within each frame (``vision_attention`` op: a HIP MFMA
  kernel on the GPU) -> proj GEMM; add+LayerNorm -> fc1 GEMM -> tanh-GELU -> fc2;
* DeepStack: after blocks ``deepstack_visual_indexes`` a merger (2x2 patch
  shuffle -> LayerNorm over 4*hidden -> fc1 -> GELU -> fc2) produces features that
  are added to the language model's hidden states at the image positions after
  decoder layers 0, 1, 2 (``LlamaModel.forward``);
* final merger (LayerNorm over hidden -> 2x2 shuffle -> fc1 -> GELU -> fc2) gives
  one language-model embedding per 2x2 patch block; those replace the embeddings of
  the ``<|image_pad|>`` tokens.

Patches arrive in 2x2-merge-block order (``multimodal.preprocess_image``), so the
shuffle is a free reshape. Behavioural reference: transformers'
``models/qwen3_vl/modeling_qwen3_vl.py`` (Qwen3VLVisionModel); parity is pinned by
``tests/test_vision.py`` against it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

from ..config import VisionConfig
from ..ops import gemm


@dataclass
class VisionBlock:
    n1w: torch.Tensor
    n1b: torch.Tensor
    qkv_w: torch.Tensor
    qkv_b: torch.Tensor
    proj_w: torch.Tensor
    proj_b: torch.Tensor
    n2w: torch.Tensor
    n2b: torch.Tensor
    fc1_w: torch.Tensor
    fc1_b: torch.Tensor
    fc2_w: torch.Tensor
    fc2_b: torch.Tensor


@dataclass
class Merger:
    nw: torch.Tensor
    nb: torch.Tensor
    fc1_w: torch.Tensor
    fc1_b: torch.Tensor
    fc2_w: torch.Tensor
    fc2_b: torch.Tensor
    post_shuffle_norm: bool = False


@dataclass
class ImageGeometry:
    """Host-side per-batch metadata of the patches of one or more images."""
    grids: list                  # [(t, h, w)] in patches
    interp_idx: np.ndarray       # int64 [Np, 4] rows of the position table
    interp_w: np.ndarray         # fp32 [Np, 4] bilinear weights
    rot_pos: np.ndarray          # int64 [Np, 2] (row, col) of each patch
    cu_seqlens: np.ndarray       # int32 [frames + 1] attention segments (one per frame)
    extra: dict = field(default_factory=dict)

    @property
    def num_patches(self) -> int:
        return int(self.cu_seqlens[-1])


def image_geometry(grids, cfg: VisionConfig) -> ImageGeometry:
    """Position-table taps, RoPE coordinates and attention segments for patches laid
    out frame by frame, each frame in 2x2-merge-block order (block row, block col,
    row in block, col in block)."""
    m = cfg.spatial_merge_size
    side = int(round(math.sqrt(cfg.num_position_embeddings)))
    idx, wts, pos, cu = [], [], [], [0]
    for t, h, w in grids:
        t, h, w = int(t), int(h), int(w)
        br, bc, ir, ic = np.meshgrid(np.arange(h // m), np.arange(w // m), np.arange(m), np.arange(m), indexing="ij")
        row = (br * m + ir).reshape(-1)
        col = (bc * m + ic).reshape(-1)
        # bilinear with aligned corners: patch r of h maps to r * (side-1) / (h-1)
        fr = row.astype(np.float64) * (side - 1) / max(h - 1, 1)
        fc = col.astype(np.float64) * (side - 1) / max(w - 1, 1)
        r0, c0 = np.floor(fr).astype(np.int64), np.floor(fc).astype(np.int64)
        r1, c1 = np.minimum(r0 + 1, side - 1), np.minimum(c0 + 1, side - 1)
        dr, dc = fr - r0, fc - c0
        ii = np.stack([r0 * side + c0, r0 * side + c1, r1 * side + c0, r1 * side + c1], 1)
        ww = np.stack([(1 - dr) * (1 - dc), (1 - dr) * dc, dr * (1 - dc), dr * dc], 1)
        for _ in range(t):
            idx.append(ii)
            wts.append(ww)
            pos.append(np.stack([row, col], 1))
            cu.append(cu[-1] + h * w)
    return ImageGeometry(list(grids), np.concatenate(idx).astype(np.int64),
                         np.concatenate(wts).astype(np.float32), np.concatenate(pos).astype(np.int64),
                         np.asarray(cu, dtype=np.int32))


def rope_table_2d(rot_pos: torch.Tensor, head_dim: int, theta: float = 10000.0) -> torch.Tensor:
    """fp32 [Np, head_dim] = [cos | sin] of the angles (row * f_i for the first
    head_dim/4 frequencies, col * f_i for the next head_dim/4), f_i = theta^(-4i/head_dim)
    (HF: rotary dim head_dim/2, each axis half of it, duplicated for rotate-half)."""
    rd = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, rd, 2, dtype=torch.float32) / rd))
    p = rot_pos.to(torch.float32)
    ang = torch.cat([p[:, :1] * inv, p[:, 1:2] * inv], 1)  # [Np, head_dim/2]
    return torch.cat([ang.cos(), ang.sin()], 1).contiguous()


class VisionTower:
    def __init__(self, cfg: VisionConfig, device, dtype, ops):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.ops = ops
        self.blocks: list[VisionBlock] = []
        self.patch_w = self.patch_b = self.pos_embed = None
        self.merger: Merger | None = None
        self.deepstack: list[Merger] = []
        self.eps = 1e-6

    # ------------------------------------------------------------ weights
    def load(self, get, prefix: str):
        """``get(name) -> tensor`` over a checkpoint; ``prefix`` e.g. "model.visual."."""
        c = self.cfg

        def t(name, dtype=None):
            return get(prefix + name).to(device=self.device, dtype=dtype or self.dtype).contiguous()

        self.patch_w = t("patch_embed.proj.weight").reshape(c.hidden_size, -1).contiguous()
        self.patch_b = t("patch_embed.proj.bias")
        self.pos_embed = t("pos_embed.weight")
        self.blocks = []
        for i in range(c.depth):
            p = f"blocks.{i}."
            self.blocks.append(VisionBlock(
                t(p + "norm1.weight"), t(p + "norm1.bias"), t(p + "attn.qkv.weight"), t(p + "attn.qkv.bias"),
                t(p + "attn.proj.weight"), t(p + "attn.proj.bias"), t(p + "norm2.weight"), t(p + "norm2.bias"),
                t(p + "mlp.linear_fc1.weight"), t(p + "mlp.linear_fc1.bias"),
                t(p + "mlp.linear_fc2.weight"), t(p + "mlp.linear_fc2.bias")))

        def merger(p, post):
            return Merger(t(p + "norm.weight"), t(p + "norm.bias"), t(p + "linear_fc1.weight"),
                          t(p + "linear_fc1.bias"), t(p + "linear_fc2.weight"), t(p + "linear_fc2.bias"), post)

        self.merger = merger("merger.", False)
        self.deepstack = [merger(f"deepstack_merger_list.{j}.", True)
                          for j in range(len(c.deepstack_visual_indexes))]

    def allocate_random(self, seed: int = 0, std: float = 0.02):
        """Random-init tower of the configured shape (benchmarks / smoke tests)."""
        c = self.cfg
        g = torch.Generator(device="cpu").manual_seed(seed + 77)
        C, I, M = c.hidden_size, c.intermediate_size, c.hidden_size * c.spatial_merge_size ** 2

        def rnd(*s):
            return (torch.randn(*s, generator=g) * std).to(device=self.device, dtype=self.dtype)

        def ones(n):
            return torch.ones(n, device=self.device, dtype=self.dtype)

        def zeros(n):
            return torch.zeros(n, device=self.device, dtype=self.dtype)

        self.patch_w, self.patch_b = rnd(C, c.patch_dim), zeros(C)
        self.pos_embed = rnd(c.num_position_embeddings, C)
        self.blocks = [VisionBlock(ones(C), zeros(C), rnd(3 * C, C), zeros(3 * C), rnd(C, C), zeros(C),
                                   ones(C), zeros(C), rnd(I, C), zeros(I), rnd(C, I), zeros(C))
                       for _ in range(c.depth)]

        def merger(post):
            return Merger(ones(M if post else C), zeros(M if post else C), rnd(M, M), zeros(M),
                          rnd(c.out_hidden_size, M), zeros(c.out_hidden_size), post)

        self.merger = merger(False)
        self.deepstack = [merger(True) for _ in c.deepstack_visual_indexes]

    # ------------------------------------------------------------ forward
    def _merge(self, x: torch.Tensor, mg: Merger) -> torch.Tensor:
        m2 = self.cfg.spatial_merge_size ** 2
        C = self.cfg.hidden_size
        if mg.post_shuffle_norm:
            y = x.reshape(-1, C * m2)
            yn = torch.empty_like(y)
            self.ops.layernorm(yn, y, mg.nw, mg.nb, self.eps)
        else:
            yn = torch.empty_like(x)
            self.ops.layernorm(yn, x, mg.nw, mg.nb, self.eps)
            yn = yn.view(-1, C * m2)
        h = F.linear(yn, mg.fc1_w, mg.fc1_b)
        self.ops.gelu_(h, False)
        return F.linear(h, mg.fc2_w, mg.fc2_b)

    @torch.inference_mode()
    def forward(self, pixels: torch.Tensor, geo: ImageGeometry):
        """pixels [Np, patch_dim] -> (embeddings [Np / merge^2, out_hidden],
        [deepstack features [Np / merge^2, out_hidden]] per deepstack index)."""
        c, ops, dev = self.cfg, self.ops, self.device
        nh, D = c.num_heads, c.head_dim
        x = F.linear(pixels.to(device=dev, dtype=self.dtype), self.patch_w, self.patch_b)
        idx = torch.from_numpy(geo.interp_idx).to(dev)
        w = torch.from_numpy(geo.interp_w).to(dev)
        pe = (self.pos_embed[idx].float() * w[..., None]).sum(1).to(self.dtype)
        x = x + pe
        cos_sin = rope_table_2d(torch.from_numpy(geo.rot_pos), D).to(dev)
        cu = torch.from_numpy(geo.cu_seqlens).to(dev)
        scale = D ** -0.5
        Np = x.shape[0]
        xn = torch.empty_like(x)
        attn = torch.empty(Np, nh * D, device=dev, dtype=self.dtype)
        meta = ops.vision_meta(geo, nh, D) if hasattr(ops, "vision_meta") else None
        ds = []
        pending = None  # residual stream update not yet added (fused into the next LayerNorm)
        for i, b in enumerate(self.blocks):
            if pending is None:
                ops.layernorm(xn, x, b.n1w, b.n1b, self.eps)
            else:
                ops.layernorm(xn, pending, b.n1w, b.n1b, self.eps, residual=x)
            qkv = F.linear(xn, b.qkv_w, b.qkv_b)
            ops.vision_attention(attn, qkv, cos_sin, cu, nh, D, scale, meta)
            o = F.linear(attn, b.proj_w, b.proj_b)
            ops.layernorm(xn, o, b.n2w, b.n2b, self.eps, residual=x)
            if xn.is_cuda and c.hidden_act in ("gelu_pytorch_tanh", "gelu_tanh"):
                # fc1 + bias + GELU in one hipBLASLt call (GELU epilogue): 228 vs 296 us
                # for GEMM + separate GELU pass at 16K patches, same error vs fp32
                h = torch._addmm_activation(b.fc1_b, xn, b.fc1_w.t(), use_gelu=True)
            else:
                h = F.linear(xn, b.fc1_w, b.fc1_b)
                ops.gelu_(h, c.hidden_act in ("gelu_pytorch_tanh", "gelu_tanh"))
            pending = F.linear(h, b.fc2_w, b.fc2_b)
            if i in c.deepstack_visual_indexes:
                x = x + pending
                pending = None
                ds.append(self._merge(x, self.deepstack[c.deepstack_visual_indexes.index(i)]))
        if pending is not None:
            x = x + pending
        return self._merge(x, self.merger), ds
