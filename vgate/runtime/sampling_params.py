"""Per-request sampling parameters for the native engine."""
from __future__ import annotations

from dataclasses import dataclass, field


@dataclass
class SamplingParams:
    temperature: float = 0.7
    top_p: float = 0.9
    top_k: int = -1
    max_tokens: int = 256
    seed: int | None = None
    stop_token_ids: list[int] = field(default_factory=list)
    stop: list[str] = field(default_factory=list)
    ignore_eos: bool = False
    min_tokens: int = 0

    def __post_init__(self):
        if self.temperature < 0:
            raise ValueError("temperature must be >= 0")
        if not (0.0 < self.top_p <= 1.0):
            raise ValueError("top_p must be in (0, 1]")
        if self.max_tokens < 1:
            raise ValueError("max_tokens must be >= 1")
        if self.top_k == 0:
            self.top_k = -1

    @property
    def greedy(self) -> bool:
        return self.temperature <= 1e-5
