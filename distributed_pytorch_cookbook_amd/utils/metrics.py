"""Throughput metrics (absent in the reference): training FLOPs per token,
model FLOP utilisation against the MI355X dense bf16 peak, and peak device memory.

FLOPs per token follow the usual 6 * (non-embedding parameters) + attention term
(6·P_nonembed + 12·L·S·D), computed for the reference architecture
(``/root/reference/models/gpt.py:10-231``: untied lm_head, Q/K/V without bias, FFN 4x).
"""
from __future__ import annotations

import torch

# AMD's dense (no 2:1 sparsity) bf16 MFMA figure for one MI355X
MI355X_BF16_DENSE_FLOPS = 2.5e15


def nonembed_params(dim: int, heads: int, head_dim: int, num_layers: int, vocab: int) -> int:
    a = heads * head_dim
    per_layer = (3 * dim * a            # to_q / to_k / to_v
                 + a * dim + dim        # to_out (+ bias)
                 + dim * 4 * dim + 4 * dim + 4 * dim * dim + dim  # up / down (+ biases)
                 + 4 * dim)             # norm1 / norm2
    return num_layers * per_layer + 2 * dim + vocab * dim  # + norm_out + lm_head


def train_flops_per_token(dim: int, heads: int, head_dim: int, num_layers: int, vocab: int,
                          seq_len: int) -> float:
    """Forward + backward FLOPs per trained token (causal attention counted in full, as
    the usual MFU convention does)."""
    return 6.0 * nonembed_params(dim, heads, head_dim, num_layers, vocab) + \
        12.0 * num_layers * seq_len * heads * head_dim


def mfu(tokens_per_s_per_gpu: float, flops_per_token: float,
        peak: float = MI355X_BF16_DENSE_FLOPS) -> float:
    return tokens_per_s_per_gpu * flops_per_token / peak


def peak_memory_gib(device) -> float:
    if torch.device(device).type != "cuda":
        return 0.0
    return torch.cuda.max_memory_allocated(device) / 2**30
