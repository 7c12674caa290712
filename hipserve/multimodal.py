"""Image inputs of the OpenAI chat surface for the Qwen3-VL vision tower.

* ``load_image``: an ``image_url`` content part (``data:`` URL with base64 payload,
  ``file://`` / local path when allowed, or http(s) with a timeout and size cap) ->
  RGB PIL image;
* ``smart_resize`` / ``preprocess_image``: resize so both sides are multiples of
  patch*merge (32) within [min_pixels, max_pixels] keeping the aspect ratio, bicubic
  resample, scale to [0, 1], normalise by mean/std, and cut into 16x16 patches laid
  out in 2x2-merge-block order with the frame repeated over the temporal patch (2) —
  the same pixel layout as the Qwen2-VL/Qwen3-VL image processor, so checkpoints
  see the inputs they were trained on (parity: tests/test_vision.py);
* ``expand_image_tokens``: each ``<|image_pad|>`` of the templated prompt becomes
  (h/2)*(w/2) copies, one per merged patch;
* ``mrope_positions``: the 3D (t, h, w) rotary positions of the prompt and the
  delta that continues text positions after it.
"""
from __future__ import annotations

import base64
import hashlib
import io
import math
import os
from dataclasses import dataclass

import numpy as np

from .config import VisionConfig

MAX_IMAGE_BYTES = 32 << 20


class ImageInputError(ValueError):
    """Unusable image content part (HTTP 400)."""


@dataclass
class ImageInput:
    pixels: np.ndarray      # fp32 [Np, patch_dim]
    grid: tuple             # (t, h, w) in patches
    digest: int             # content hash (prefix-cache key of the image tokens)

    @property
    def num_tokens(self) -> int:
        t, h, w = self.grid
        return t * h * w // 4


@dataclass
class MultiModalPrompt:
    """A tokenised prompt whose image placeholders are already expanded, with its images."""
    ids: list
    images: list


@dataclass
class MMState:
    """Per-sequence multimodal state (engine side)."""
    images: list            # [ImageInput]
    spans: list             # [(start, end)] token range of each image
    pos3: np.ndarray        # int64 [3, n_prompt] MRoPE positions
    delta: int              # rotary position of token i >= n_prompt is i + delta
    hash_ids: list          # prompt ids with image tokens replaced by content-keyed ids (< 0)


def mm_state(ids: list[int], images: list, cfg: VisionConfig) -> MMState:
    spans = image_spans(ids, images, cfg)
    pos3, delta = mrope_positions(len(ids), spans, images, cfg.spatial_merge_size)
    hids = list(ids)
    for (a, b), im in zip(spans, images):
        for j in range(a, b):  # negative ids never collide with vocabulary ids
            hids[j] = -1 - ((im.digest + 0x9E3779B97F4A7C15 * (j - a + 1)) & 0x3FFFFFFF)
    return MMState(images, spans, pos3, delta, hids)


def load_image(url: str, allow_local: bool = False, timeout: float = 10.0):
    from PIL import Image

    if not isinstance(url, str) or not url:
        raise ImageInputError("image_url.url must be a non-empty string")
    if url.startswith("data:"):
        head, _, payload = url.partition(",")
        if ";base64" not in head:
            raise ImageInputError("data: image URLs must be base64-encoded")
        try:
            data = base64.b64decode(payload, validate=False)
        except (ValueError, TypeError) as e:
            raise ImageInputError(f"bad base64 image payload: {e}") from None
    elif url.startswith(("http://", "https://")):
        import urllib.request

        try:
            with urllib.request.urlopen(url, timeout=timeout) as r:  # noqa: S310 (scheme checked)
                data = r.read(MAX_IMAGE_BYTES + 1)
        except OSError as e:
            raise ImageInputError(f"could not fetch image {url!r}: {e}") from None
    elif allow_local and (url.startswith("file://") or os.path.isabs(url)):
        path = url[len("file://"):] if url.startswith("file://") else url
        try:
            with open(path, "rb") as f:
                data = f.read(MAX_IMAGE_BYTES + 1)
        except OSError as e:
            raise ImageInputError(f"could not read image {path!r}: {e}") from None
    else:
        raise ImageInputError("image_url must be a data: URL or an http(s) URL")
    if len(data) > MAX_IMAGE_BYTES:
        raise ImageInputError(f"image larger than {MAX_IMAGE_BYTES} bytes")
    try:
        img = Image.open(io.BytesIO(data))
        img.load()
    except Exception as e:  # PIL raises many types on bad data
        raise ImageInputError(f"cannot decode image: {e}") from None
    return img.convert("RGB")


def smart_resize(h: int, w: int, factor: int, min_pixels: int, max_pixels: int) -> tuple[int, int]:
    if min(h, w) <= 0:
        raise ImageInputError("empty image")
    if max(h, w) / min(h, w) > 200:
        raise ImageInputError("image aspect ratio must be below 200")
    hb, wb = round(h / factor) * factor, round(w / factor) * factor
    if hb * wb > max_pixels:
        beta = math.sqrt(h * w / max_pixels)
        hb = max(factor, math.floor(h / beta / factor) * factor)
        wb = max(factor, math.floor(w / beta / factor) * factor)
    elif hb * wb < min_pixels:
        beta = math.sqrt(min_pixels / (h * w))
        hb = math.ceil(h * beta / factor) * factor
        wb = math.ceil(w * beta / factor) * factor
    return hb, wb


def preprocess_image(img, cfg: VisionConfig, max_pixels: int | None = None) -> ImageInput:
    from PIL import Image

    p, m, tp = cfg.patch_size, cfg.spatial_merge_size, cfg.temporal_patch_size
    W0, H0 = img.size
    H, W = smart_resize(H0, W0, p * m, cfg.min_pixels, max_pixels or cfg.max_pixels)
    if (W, H) != (W0, H0):
        img = img.resize((W, H), resample=Image.BICUBIC)
    a = np.asarray(img, dtype=np.uint8).astype(np.float32) * np.float32(1 / 255)
    a = (a - np.asarray(cfg.image_mean, np.float32)) / np.asarray(cfg.image_std, np.float32)
    a = a.transpose(2, 0, 1)  # C, H, W
    C = a.shape[0]
    gh, gw = H // p, W // p
    x = a.reshape(C, gh // m, m, p, gw // m, m, p).transpose(1, 4, 2, 5, 0, 3, 6)  # bh bw mh mw C ph pw
    x = np.broadcast_to(x[:, :, :, :, :, None], (*x.shape[:5], tp, p, p))
    pix = np.ascontiguousarray(x.reshape(gh * gw, C * tp * p * p), dtype=np.float32)
    digest = int.from_bytes(hashlib.blake2b(pix.tobytes(), digest_size=8).digest(), "little")
    return ImageInput(pix, (1, gh, gw), digest)


def expand_image_tokens(ids: list[int], images: list[ImageInput], cfg: VisionConfig) -> list[int]:
    """Replace the i-th ``<|image_pad|>`` with images[i].num_tokens copies (the chat
    template emits one per image part)."""
    out, k = [], 0
    for t in ids:
        if t == cfg.image_token_id:
            if k >= len(images):
                raise ImageInputError("more image placeholders than images")
            out.extend([t] * images[k].num_tokens)
            k += 1
        else:
            out.append(t)
    if k != len(images):
        raise ImageInputError(f"{len(images)} images but {k} image placeholders in the prompt")
    return out


def image_spans(ids: list[int], images: list[ImageInput], cfg: VisionConfig) -> list[tuple[int, int]]:
    """[start, end) token range of each image in an expanded prompt."""
    spans, i, k, n = [], 0, 0, len(ids)
    while i < n:
        if ids[i] == cfg.image_token_id:
            if k >= len(images):
                raise ImageInputError("more image tokens than images")
            e = i + images[k].num_tokens
            if e > n or any(t != cfg.image_token_id for t in ids[i:e]):
                raise ImageInputError("image token run does not match the image size")
            spans.append((i, e))
            i, k = e, k + 1
        else:
            i += 1
    if k != len(images):
        raise ImageInputError(f"{len(images)} images but {k} image token runs in the prompt")
    return spans


def mrope_positions(n: int, spans: list[tuple[int, int]], images: list[ImageInput], merge: int = 2):
    """(int64 [3, n] (t, h, w) rotary positions of an n-token prompt, delta) — text
    tokens advance all three axes together; an image's tokens sit on its merged grid
    offset by the running position, after which text resumes at that offset plus
    max(h, w)/merge. Tokens appended later use position index + delta on all axes."""
    pos = np.empty((3, n), np.int64)
    cur, i = 0, 0
    for (a, b), im in zip(spans, images):
        L = a - i
        pos[:, i:a] = cur + np.arange(L)
        cur += L
        t, h, w = im.grid
        gh, gw = h // merge, w // merge
        tt, hh, ww = np.meshgrid(np.arange(t), np.arange(gh), np.arange(gw), indexing="ij")
        pos[0, a:b] = tt.reshape(-1) + cur
        pos[1, a:b] = hh.reshape(-1) + cur
        pos[2, a:b] = ww.reshape(-1) + cur
        cur += max(gh, gw)
        i = b
    pos[:, i:] = cur + np.arange(n - i)
    delta = int(pos.max()) + 1 - n if n else 0
    return pos, delta


def mrope_cos_sin(pos3: np.ndarray, head_dim: int, theta: float, section) -> np.ndarray:
    """fp32 [n, head_dim] [cos | sin] rows of interleaved MRoPE: rotary pair j uses the
    h position when j % 3 == 1 and j < 3*section[1], the w position when j % 3 == 2 and
    j < 3*section[2], else t (Qwen3-VL ``apply_interleaved_mrope``)."""
    half = head_dim // 2
    inv = 1.0 / (theta ** (np.arange(0, head_dim, 2, dtype=np.float64) / head_dim))
    axis = np.zeros(half, np.int64)
    j = np.arange(half)
    axis[(j % 3 == 1) & (j < 3 * section[1])] = 1
    axis[(j % 3 == 2) & (j < 3 * section[2])] = 2
    p = pos3[axis].astype(np.float64).T  # [n, half]
    ang = p * inv
    return np.concatenate([np.cos(ang), np.sin(ang)], 1).astype(np.float32)
