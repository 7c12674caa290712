"""Tokenizers: HF ``tokenizer.json`` (HF tier), GGUF-embedded vocab (GGUF tier,
see ``hipserve.weights.gguf``) and a synthetic byte-level tokenizer for
random-init benchmark models (no network => no Hub tokenizer)."""
from __future__ import annotations

import json
import os

_DEFAULT_CHAT_TEMPLATE = (
    "{{ bos_token }}{% for m in messages %}<|start_header_id|>{{ m['role'] }}<|end_header_id|>\n\n"
    "{{ m['content'] }}<|eot_id|>{% endfor %}"
    "{% if add_generation_prompt %}<|start_header_id|>assistant<|end_header_id|>\n\n{% endif %}")


class UnsupportedContentError(ValueError):
    """An OpenAI content part the served model cannot consume (HTTP 400)."""


def render_chat(template: str, messages: list[dict], bos_token: str = "", eos_token: str = "",
                add_generation_prompt: bool = True) -> str:
    import jinja2

    env = jinja2.Environment(trim_blocks=True, lstrip_blocks=True)

    def raise_exception(msg):
        raise ValueError(msg)

    env.globals["raise_exception"] = raise_exception
    msgs = []
    for m in messages:
        if not isinstance(m, dict):
            raise ValueError("each message must be an object with 'role' and 'content'")
        c = m.get("content", "")
        if c is None:
            c = ""
        if isinstance(c, list):  # OpenAI content parts: text only (no vision tower is served)
            for p in c:
                if not isinstance(p, dict) or p.get("type", "text") != "text":
                    kind = p.get("type") if isinstance(p, dict) else type(p).__name__
                    raise UnsupportedContentError(
                        f"content part of type {kind!r} is not supported: this deployment serves the "
                        "model's text path only (image / audio inputs are rejected, not dropped)")
            c = "".join(p.get("text", "") for p in c)
        elif not isinstance(c, str):
            raise ValueError("message content must be a string or a list of content parts")
        msgs.append({**m, "content": c})
    return env.from_string(template).render(messages=msgs, bos_token=bos_token, eos_token=eos_token,
                                            add_generation_prompt=add_generation_prompt)


class BaseTokenizer:
    bos_token_id: int | None = None
    eos_token_ids: tuple = ()
    bos_token: str = ""
    eos_token: str = ""
    chat_template: str = _DEFAULT_CHAT_TEMPLATE
    vocab_size: int = 0
    add_bos: bool = True
    chat_adds_bos: bool = True

    def encode(self, text: str, add_special_tokens: bool = True) -> list[int]:
        raise NotImplementedError

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        raise NotImplementedError

    def apply_chat_template(self, messages, add_generation_prompt=True) -> str:
        return render_chat(self.chat_template, messages, self.bos_token, self.eos_token,
                           add_generation_prompt)

    def encode_chat(self, messages, add_generation_prompt=True) -> list[int]:
        text = self.apply_chat_template(messages, add_generation_prompt)
        ids = self.encode(text, add_special_tokens=False)
        if self.bos_token_id is not None and self.add_bos and (not ids or ids[0] != self.bos_token_id) \
                and not self.bos_token:
            ids = [self.bos_token_id] + ids
        return ids

    def encode_chat_mm(self, messages, vision) -> tuple[list[int], list[str]]:
        """Chat prompt of a vision model: every image part (OpenAI ``image_url`` or
        ``image``) becomes ``<|vision_start|><|image_pad|><|vision_end|>`` — what the
        Qwen3-VL chat template emits for it — and its URL is returned, in prompt order.
        The single ``<|image_pad|>`` per image is expanded by the caller once the
        image's patch grid is known. Text segments are tokenised separately around the
        image markers, so tokenizers without these special tokens work too."""
        urls: list[str] = []
        flat = []
        for m in messages:
            if isinstance(m, dict) and isinstance(m.get("content"), list):
                parts = []
                for p in m["content"]:
                    kind = p.get("type", "text") if isinstance(p, dict) else None
                    if kind == "text":
                        parts.append(p.get("text", ""))
                    elif kind in ("image_url", "image"):
                        u = p.get("image_url", p.get("image"))
                        u = u.get("url") if isinstance(u, dict) else u
                        urls.append(u)
                        parts.append(_IMAGE_MARK)
                    else:
                        raise UnsupportedContentError(f"content part of type {kind!r} is not supported "
                                                      "(text and image_url parts are)")
                m = {**m, "content": "".join(parts)}
            flat.append(m)
        text = self.apply_chat_template(flat, True)
        pieces = text.split(_IMAGE_MARK)
        ids = []
        for i, piece in enumerate(pieces):
            if i:
                ids += [vision.vision_start_token_id, vision.image_token_id, vision.vision_end_token_id]
            if piece:
                ids += self.encode(piece, add_special_tokens=False)
        if self.chat_adds_bos and self.bos_token_id is not None and self.add_bos \
                and (not ids or ids[0] != self.bos_token_id) and not self.bos_token:
            ids = [self.bos_token_id] + ids
        return ids, urls


_IMAGE_MARK = "<|vision_start|><|image_pad|><|vision_end|>"


class SyntheticTokenizer(BaseTokenizer):
    """Byte-level tokenizer for random-init models: ids [base, base+256) are raw
    bytes, everything else decodes to a short placeholder word."""

    def __init__(self, vocab_size: int, bos: int | None = 1, eos=(2,)):
        self.vocab_size = vocab_size
        self.bos_token_id = bos
        self.eos_token_ids = tuple(eos)
        self.special = {i for i in (bos, *self.eos_token_ids) if i is not None}
        self.base = 3 if vocab_size > 300 else 0

    def encode(self, text: str, add_special_tokens: bool = True) -> list[int]:
        ids = [self.base + b for b in text.encode("utf-8")]
        ids = [i % self.vocab_size for i in ids]
        if add_special_tokens and self.bos_token_id is not None:
            ids = [self.bos_token_id] + ids
        return ids

    def decode(self, ids, skip_special_tokens: bool = True) -> str:
        out = bytearray()
        words = []
        for i in ids:
            i = int(i)
            if i in self.special:
                if not skip_special_tokens:
                    out += f"<s{i}>".encode()
                continue
            if self.base <= i < self.base + 256:
                out.append(i - self.base)
            else:
                out += f" w{i}".encode()
        return out.decode("utf-8", errors="replace") + "".join(words)


class HFTokenizer(BaseTokenizer):
    """``tokenizers`` fast tokenizer loaded from a local model directory."""

    def __init__(self, path: str, eos_fallback=()):
        from tokenizers import Tokenizer

        self.tk = Tokenizer.from_file(os.path.join(path, "tokenizer.json"))
        self.vocab_size = self.tk.get_vocab_size(with_added_tokens=True)
        cfg = {}
        p = os.path.join(path, "tokenizer_config.json")
        if os.path.exists(p):
            with open(p) as f:
                cfg = json.load(f)

        def tok_str(x):
            if isinstance(x, dict):
                return x.get("content", "")
            return x or ""

        self.bos_token = tok_str(cfg.get("bos_token"))
        self.eos_token = tok_str(cfg.get("eos_token"))
        self.bos_token_id = self.tk.token_to_id(self.bos_token) if self.bos_token else None
        eos = self.tk.token_to_id(self.eos_token) if self.eos_token else None
        ids = {e for e in (eos, *eos_fallback) if e is not None}
        self.eos_token_ids = tuple(sorted(ids))
        tmpl = cfg.get("chat_template")
        if isinstance(tmpl, list):
            tmpl = next((t["template"] for t in tmpl if t.get("name") == "default"), tmpl[0]["template"])
        if tmpl:
            self.chat_template = tmpl
        self.add_bos = cfg.get("add_bos_token", True)

    def encode(self, text, add_special_tokens=True):
        return self.tk.encode(text, add_special_tokens=add_special_tokens).ids

    def decode(self, ids, skip_special_tokens=True):
        return self.tk.decode(list(ids), skip_special_tokens=skip_special_tokens)

    def encode_chat(self, messages, add_generation_prompt=True):
        text = self.apply_chat_template(messages, add_generation_prompt)
        return self.tk.encode(text, add_special_tokens=False).ids

    chat_adds_bos = False  # HF chat templates carry any BOS themselves


def get_tokenizer(model: str, model_cfg, tokenizer: str | None = None) -> BaseTokenizer:
    path = tokenizer or model
    if os.path.isdir(path) and os.path.exists(os.path.join(path, "tokenizer.json")):
        return HFTokenizer(path, eos_fallback=model_cfg.eos_token_id)
    if path.endswith(".gguf") and os.path.exists(path):
        from ..weights.gguf import GGUFFile, GGUFTokenizer

        return GGUFTokenizer(GGUFFile(path))
    from ..config import _hf_cache_dir

    hub = _hf_cache_dir(path)
    if hub and os.path.exists(os.path.join(hub, "tokenizer.json")):
        return HFTokenizer(hub, eos_fallback=model_cfg.eos_token_id)
    return SyntheticTokenizer(model_cfg.vocab_size, model_cfg.bos_token_id, model_cfg.eos_token_id)


class IncrementalDetokenizer:
    """Streams text for a growing id list without re-decoding everything and
    without emitting partial UTF-8 sequences (prefix/read offset scheme)."""

    def __init__(self, tokenizer: BaseTokenizer, prompt_tail: list[int] | None = None):
        self.tk = tokenizer
        self.ids: list[int] = list(prompt_tail or [])[-4:]
        self.prefix_offset = len(self.ids)
        self.read_offset = len(self.ids)

    def add(self, new_ids: list[int]) -> str:
        self.ids.extend(new_ids)
        prefix = self.tk.decode(self.ids[self.prefix_offset:self.read_offset])
        full = self.tk.decode(self.ids[self.prefix_offset:])
        if len(full) > len(prefix) and not full.endswith("�"):
            self.prefix_offset = self.read_offset
            self.read_offset = len(self.ids)
            return full[len(prefix):]
        return ""
