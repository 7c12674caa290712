"""Sequence-level view of the native paged-KV block pool (csrc/runtime/block_pool.cpp)."""
from __future__ import annotations

from ..runtime import native
from .request import Sequence


def _hash_prompt(seq: Sequence) -> list[int]:
    """Prompt ids as prefix-cache keys: image placeholder tokens are keyed by their
    image's content (two prompts with different images never share KV blocks)."""
    return seq.mm.hash_ids if seq.mm is not None else seq.prompt_token_ids


class BlockManager:
    def __init__(self, num_blocks: int, block_size: int, prefix_caching: bool = True,
                 watermark: float = 0.01):
        self.block_size = block_size
        self.pool = native().BlockPool(num_blocks, block_size, prefix_caching)
        self.prefix_caching = prefix_caching
        self.watermark_blocks = max(1, int(watermark * num_blocks))
        self.num_blocks = num_blocks
        self.prefix_hit_tokens = 0
        self.prefix_query_tokens = 0

    def num_free(self) -> int:
        return self.pool.num_free()

    def usage(self) -> float:
        return self.pool.usage()

    def needed(self, seq: Sequence, target_tokens: int) -> int:
        return max(0, -(-target_tokens // self.block_size) - len(seq.block_ids))

    def can_grow(self, seq: Sequence, target_tokens: int, watermark: bool = False) -> bool:
        free = self.pool.num_free() - (self.watermark_blocks if watermark else 0)
        return self.needed(seq, target_tokens) <= free

    def grow(self, seq: Sequence, target_tokens: int):
        n = self.needed(seq, target_tokens)
        if n:
            seq.block_ids.extend(self.pool.allocate(n))

    def match_prefix(self, seq: Sequence):
        if not self.prefix_caching:
            return
        ids, ntok = self.pool.match_prefix(_hash_prompt(seq) + seq.output_token_ids)
        seq.block_ids = list(ids)
        seq.num_computed_tokens = ntok
        seq.num_cached_prefix = ntok
        self.prefix_hit_tokens += ntok
        self.prefix_query_tokens += seq.num_tokens

    def register(self, seq: Sequence):
        """Publish the sequence's completely filled blocks to the prefix cache."""
        if not self.prefix_caching:
            return
        bs = self.block_size
        full = seq.num_computed_tokens // bs
        first = getattr(seq, "_registered_blocks", 0)
        if full > first:
            # only the newly filled blocks' tokens, hash chained from the last call
            # (O(new tokens) per step, not O(context))
            a, b, npr = first * bs, full * bs, seq.num_prompt_tokens
            prompt = _hash_prompt(seq)
            toks = prompt[a:b] if b <= npr else (prompt[a:] + seq.output_token_ids[max(0, a - npr):b - npr])
            seq._reg_hash = self.pool.register_blocks(seq.block_ids, toks, first, full,
                                                       getattr(seq, "_reg_hash", 0) if first else 0)
            seq._registered_blocks = full

    def free(self, seq: Sequence):
        if seq.block_ids:
            self.pool.free(seq.block_ids)
        seq.block_ids = []
        seq._registered_blocks = 0

    def reset_prefix_cache(self):
        self.pool.reset_prefix_cache()
