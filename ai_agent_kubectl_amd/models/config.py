"""Model architecture presets (public HF configs; SURVEY.md §2.4 'Model constants').

The reference has no model code at all — its model is remote (`/root/reference/app.py:117`).
These are the architectures BASELINE.json names for the on-node engine, plus tiny variants of the
same shape family used by CPU tests and GPU numerics tests.
"""
from __future__ import annotations

import dataclasses
from typing import Dict


@dataclasses.dataclass(frozen=True)
class ModelConfig:
    name: str
    family: str                 # "llama" | "mixtral"
    num_layers: int
    hidden: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate: int
    vocab_size: int
    rope_theta: float
    norm_eps: float = 1e-5
    max_position: int = 8192
    num_experts: int = 0        # mixtral
    top_k: int = 0
    tie_embeddings: bool = False
    tokenizer: str = "llama3"   # "llama3" | "llama2"

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def num_params(self) -> int:
        h, i, v = self.hidden, self.intermediate, self.vocab_size
        attn = h * self.qkv_size + self.q_size * h
        mlp = 3 * h * i * (self.num_experts if self.is_moe else 1) + (h * self.num_experts if self.is_moe else 0)
        per_layer = attn + mlp + 2 * h
        return self.num_layers * per_layer + v * h * (1 if self.tie_embeddings else 2) + h

    def default_step_tokens(self) -> int:
        """Engine token budget per step when MAX_NUM_BATCHED_TOKENS is 0 (auto).  Each step streams
        every weight once, so a step has a fixed cost that grows with the model: for an 8B model a
        256-request wave's ~8k prompt tokens are best split over ~3 mixed steps that also carry the
        running decodes (4096: 1243-1273 vs 1109-1122 req/s at 16384), while Mixtral-8x7B and
        Llama-3-70B do better with the wave's prompt in one step (16384: 269 vs 252 and 102 vs 91
        req/s; profiles/r2/budget/)."""
        return 4096 if self.num_params() * 2 < (40 << 30) else 16384

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return self.num_layers * 2 * self.kv_size * dtype_bytes


PRESETS: Dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig("llama3-8b", "llama", 32, 4096, 32, 8, 128, 14336, 128256, 500000.0),
    "llama3-70b": ModelConfig("llama3-70b", "llama", 80, 8192, 64, 8, 128, 28672, 128256, 500000.0),
    "mixtral-8x7b": ModelConfig("mixtral-8x7b", "mixtral", 32, 4096, 32, 8, 128, 14336, 32000, 1e6,
                                max_position=32768, num_experts=8, top_k=2, tokenizer="llama2"),
    # Same shape family, small enough for CPU tests (fp32 reference) and quick GPU numerics.
    "tiny-llama": ModelConfig("tiny-llama", "llama", 2, 256, 4, 2, 64, 512, 128256, 500000.0),
    "tiny-mixtral": ModelConfig("tiny-mixtral", "mixtral", 2, 256, 4, 2, 64, 384, 32000, 1e6, num_experts=4,
                                top_k=2, tokenizer="llama2"),
    # GPU test model with the real head geometry (head_dim 128, GQA 4) but few layers.
    "llama3-8b-2l": ModelConfig("llama3-8b-2l", "llama", 2, 4096, 32, 8, 128, 14336, 128256, 500000.0),
    # Llama-3-70B geometry (8 KV heads: 1 per rank at TP = 8, GQA group 8) with 2 layers: TP = 4 / 8
    # numerics on one GPU (tests/virtual_tp.py, tests/test_tp_single_gpu.py)
    "llama3-70b-2l": ModelConfig("llama3-70b-2l", "llama", 2, 8192, 64, 8, 128, 28672, 128256, 500000.0),
    # 8 layers of Llama-3-70B: timing a TP group's decode step on one GPU (scripts/bench_tp_persistent_2rank.py)
    "llama3-70b-8l": ModelConfig("llama3-70b-8l", "llama", 8, 8192, 64, 8, 128, 28672, 128256, 500000.0),
    # Llama-3-70B head layout (64 q / 8 kv heads: GQA 8, one KV head per rank at TP = 8) on small
    # layers: CPU multi-process TP = 8 serving tests (gloo), where the 8192-wide layers would not fit
    "llama3-70b-tiny": ModelConfig("llama3-70b-tiny", "llama", 2, 2048, 64, 8, 32, 1024, 128256, 500000.0),
    "mixtral-2l": ModelConfig("mixtral-2l", "mixtral", 2, 4096, 32, 8, 128, 14336, 32000, 1e6, max_position=32768,
                              num_experts=8, top_k=2, tokenizer="llama2"),
}


def get_config(name: str) -> ModelConfig:
    try:
        return PRESETS[name]
    except KeyError:
        raise ValueError(f"unknown MODEL {name!r}; choose from {sorted(PRESETS)}") from None
