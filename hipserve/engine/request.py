"""Request / sequence state and sampling parameters (OpenAI request surface)."""
from __future__ import annotations

import enum
import time
from dataclasses import dataclass, field


@dataclass
class SamplingParams:
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    max_tokens: int = 16
    min_tokens: int = 0
    stop: list[str] = field(default_factory=list)
    stop_token_ids: list[int] = field(default_factory=list)
    ignore_eos: bool = False
    seed: int | None = None
    presence_penalty: float = 0.0
    frequency_penalty: float = 0.0
    repetition_penalty: float = 1.0
    logprobs: int | None = None
    n: int = 1

    def __post_init__(self):
        if isinstance(self.stop, str):
            self.stop = [self.stop]
        self.stop = list(self.stop or [])
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not 0.0 < self.top_p <= 1.0:
            raise ValueError("top_p must be in (0, 1]")
        if self.max_tokens is not None and self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if self.top_k < 0:
            self.top_k = 0

    @property
    def greedy(self) -> bool:
        return self.temperature <= 1e-5

    @property
    def has_penalties(self) -> bool:
        return (self.presence_penalty != 0.0 or self.frequency_penalty != 0.0
                or self.repetition_penalty != 1.0)


class Status(enum.Enum):
    WAITING = 0
    RUNNING = 1
    PREEMPTED = 2
    FINISHED = 3


@dataclass
class Sequence:
    request_id: str
    prompt_token_ids: list[int]
    params: SamplingParams
    eos_token_ids: tuple = ()
    arrival_time: float = field(default_factory=time.monotonic)
    output_token_ids: list[int] = field(default_factory=list)
    output_logprobs: list[float] = field(default_factory=list)
    status: Status = Status.WAITING
    block_ids: list[int] = field(default_factory=list)
    num_computed_tokens: int = 0        # tokens whose KV is in the cache
    num_cached_prefix: int = 0          # tokens served from the prefix cache
    finish_reason: str | None = None
    stop_reason: object = None
    first_token_time: float | None = None
    last_token_time: float | None = None
    seed: int = 0
    # detokenizer state
    output_text: str = ""
    _decoded_upto: int = 0
    _prefix_offset: int = 0
    _read_offset: int = 0

    @property
    def num_tokens(self) -> int:
        return len(self.prompt_token_ids) + len(self.output_token_ids)

    @property
    def num_prompt_tokens(self) -> int:
        return len(self.prompt_token_ids)

    def all_token_ids(self) -> list[int]:
        return self.prompt_token_ids + self.output_token_ids

    def token_at(self, i: int) -> int:
        n = len(self.prompt_token_ids)
        return self.prompt_token_ids[i] if i < n else self.output_token_ids[i - n]

    @property
    def num_uncomputed(self) -> int:
        return self.num_tokens - self.num_computed_tokens

    @property
    def is_prefill(self) -> bool:
        """True while prompt (or recomputed) tokens remain; decode = exactly the
        last sampled token is missing from the KV cache."""
        return self.num_uncomputed > 1 or not self.output_token_ids

    @property
    def finished(self) -> bool:
        return self.status == Status.FINISHED


@dataclass
class RequestOutput:
    request_id: str
    new_token_ids: list[int]
    new_text: str
    finished: bool
    finish_reason: str | None = None
    num_prompt_tokens: int = 0
    num_output_tokens: int = 0
    logprobs: list[float] | None = None
    text: str = ""
