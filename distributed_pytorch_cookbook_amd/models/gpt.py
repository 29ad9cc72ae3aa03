"""GPT-style decoder LM -- the ``models.gpt`` definition of the cookbook.

Module tree, constructor signatures, submodule names and therefore the state_dict keys
are those of ``/root/reference/models/gpt.py`` (13 tensors per layer + 5 global, see
SURVEY.md §2.2), with the reference's two crash bugs fixed (``Embeddings`` used
``self.dim`` before assignment, ``gpt.py:177``; ``forward`` used an undefined ``x``,
``gpt.py:227``) and its semantics kept, including the quirk that ``FeedForward``
applies the activation after BOTH projections (``gpt.py:34-38``, ReLU by default).

Each module's own ``forward`` is the reference math in plain torch ops (used by the
parity tests and available to users who call submodules directly).  The LM's
``forward`` runs the fused execution path (``models/fused.py``): per-layer autograd
functions driving the gfx950 kernels (MFMA GEMMs with fused bias/activation/residual
epilogues, flash attention, fused LayerNorm, fused cross-entropy), with weights and
gradients living in flat buffers owned by a parameter store (``parallel/store.py``) so
that DDP / FSDP / pipeline engines can bucket, shard and overlap communication.
"""
from __future__ import annotations

from math import sqrt
from typing import Callable, Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

ACTIVATIONS = {"relu": F.relu, "gelu": lambda x: F.gelu(x, approximate="tanh")}


def activation_name(fn) -> str:
    if isinstance(fn, str):
        return fn
    for k, v in ACTIVATIONS.items():
        if fn is v:
            return k
    if fn is F.relu:
        return "relu"
    if fn is F.gelu:
        return "gelu"
    raise ValueError(f"unsupported activation {fn}")


class SiteDropout(nn.Dropout):
    """``nn.Dropout`` whose mask can be pinned to the fused path's counter-based mask.

    With ``spec`` unset it is ``nn.Dropout``.  ``TransformerDecoderLM.reference_forward(...,
    dropout_seed=s)`` sets ``spec`` to the same :class:`DropSpec` the fused kernels use for
    seed ``s``, so the reference math and the fused path drop identical elements.
    """

    spec = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.spec is None or not self.training:
            return super().forward(x)
        from ..ops.dropout import keep_mask

        flat = x.reshape(-1, x.shape[-1])
        return (flat * keep_mask(self.spec, flat.shape[0], flat.shape[1], x.device).to(x.dtype)).reshape(x.shape)


class FeedForward(nn.Module):
    """x -> up_proj -> act -> down_proj -> act -> dropout (reference gpt.py:10-41)."""

    def __init__(self, dim: int, mult: int = 4, activation: Callable = F.relu,
                 out_dim: Optional[int] = None, bias: bool = True, dropout: float = 0.0):
        super().__init__()
        self.dim = dim
        self.mult = mult
        self.activation = ACTIVATIONS[activation] if isinstance(activation, str) else activation
        self.out_dim = dim if out_dim is None else out_dim
        self.bias = bias
        self.up_proj = nn.Linear(dim, dim * mult, bias=bias)
        self.down_proj = nn.Linear(dim * mult, self.out_dim, bias=bias)
        self.dropout = SiteDropout(dropout)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.activation(self.up_proj(x))
        x = self.activation(self.down_proj(x))
        return self.dropout(x)


class SelfAttention(nn.Module):
    """Multi-head causal self-attention (reference gpt.py:44-105)."""

    def __init__(self, dim: int, head_dim: int, heads: int, qkv_bias: bool = False,
                 dropout: float = 0.0):
        super().__init__()
        self.dim = dim
        self.head_dim = head_dim
        self.heads = heads
        self.qkv_bias = qkv_bias
        self.to_q = nn.Linear(dim, head_dim * heads, bias=qkv_bias)
        self.to_k = nn.Linear(dim, head_dim * heads, bias=qkv_bias)
        self.to_v = nn.Linear(dim, head_dim * heads, bias=qkv_bias)
        self.to_out = nn.Linear(head_dim * heads, dim, bias=True)
        self.dropout = SiteDropout(dropout)
        self.attn_scale = 1 / sqrt(head_dim)

    def forward(self, x: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        N, S, _ = x.shape
        q = self.to_q(x).view(N, S, self.heads, self.head_dim).transpose(1, 2)
        k = self.to_k(x).view(N, S, self.heads, self.head_dim).transpose(1, 2)
        v = self.to_v(x).view(N, S, self.heads, self.head_dim).transpose(1, 2)
        logits = (q @ k.transpose(-1, -2)) * self.attn_scale
        causal = torch.ones(S, S, dtype=torch.bool, device=x.device).tril()
        logits = logits.masked_fill(~causal, -1e9)
        if mask is not None:
            logits = logits.masked_fill(mask[:, None, None, :], torch.finfo(logits.dtype).min)
        scores = F.softmax(logits.float(), dim=-1).to(v.dtype)
        out = (scores @ v).transpose(1, 2).reshape(N, S, self.heads * self.head_dim)
        return self.dropout(self.to_out(out))


class DecoderLayer(nn.Module):
    """Pre-LN block: x += attn(norm1(x)); x += fc(norm2(x)) (reference gpt.py:108-135)."""

    def __init__(self, dim: int, head_dim: int, heads: int, dropout: float = 0.0,
                 activation: Callable = F.relu):
        super().__init__()
        self.dim = dim
        self.head_dim = head_dim
        self.heads = heads
        self.attn = SelfAttention(dim=dim, head_dim=head_dim, heads=heads, dropout=dropout)
        self.norm1 = nn.LayerNorm(dim)
        self.fc = FeedForward(dim=dim, dropout=dropout, activation=activation)
        self.norm2 = nn.LayerNorm(dim)

    def forward(self, x: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        x = self.attn(self.norm1(x), mask) + x
        x = self.fc(self.norm2(x)) + x
        return x


class TransformerDecoder(nn.Module):
    def __init__(self, dim: int, head_dim: int, heads: int, num_layers: int, dropout: float = 0.0,
                 activation: Callable = F.relu):
        super().__init__()
        self.dim = dim
        self.head_dim = head_dim
        self.heads = heads
        self.num_layers = num_layers
        self.layers = nn.ModuleList([
            DecoderLayer(dim=dim, head_dim=head_dim, heads=heads, dropout=dropout, activation=activation)
            for _ in range(num_layers)
        ])

    def forward(self, x: torch.Tensor, mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        for layer in self.layers:
            x = layer(x, mask)
        return x


class Embeddings(nn.Module):
    def __init__(self, dim: int, vocab_size: int, max_position_embeddings: int):
        super().__init__()
        self.dim = dim  # reference bug gpt.py:177 fixed: set before use
        self.input_embeddings = nn.Embedding(vocab_size, dim)
        self.position_embeddings = nn.Embedding(max_position_embeddings, dim)

    def forward(self, input_ids: torch.Tensor, position_ids: torch.Tensor) -> torch.Tensor:
        return self.input_embeddings(input_ids) + self.position_embeddings(position_ids)


class TransformerDecoderLM(nn.Module):
    """Token + position embeddings -> L pre-LN decoder layers -> LayerNorm -> untied lm_head.

    ``forward(input_ids, position_ids, mask=None)`` returns logits ``[N, S, V]`` exactly
    like the reference.  ``forward(..., targets=t)`` returns a :class:`LMOutput` with the
    mean cross-entropy (ignore_index -100) computed by the fused head (the logits are
    never materialised in f32), which is what the trainers use.
    """

    def __init__(self, dim: int, head_dim: int, heads: int, num_layers: int, vocab_size: int,
                 max_position_embeddings: int, dropout: float = 0.0, activation="relu"):
        super().__init__()
        self.dim = dim
        self.head_dim = head_dim
        self.heads = heads
        self.num_layers = num_layers
        self.vocab_size = vocab_size
        self.max_position_embeddings = max_position_embeddings
        self.dropout = dropout
        self.activation = activation_name(activation)
        act_fn = ACTIVATIONS[self.activation]
        self.embeddings = Embeddings(dim=dim, vocab_size=vocab_size,
                                     max_position_embeddings=max_position_embeddings)
        self.decoder = TransformerDecoder(num_layers=num_layers, dim=dim, head_dim=head_dim,
                                          heads=heads, dropout=dropout, activation=act_fn)
        self.norm_out = nn.LayerNorm(dim)
        self.lm_head = nn.Linear(dim, vocab_size, bias=False)
        # flat-layout hint: reserve zero rows up to a multiple of 64 after the head matrix
        # (parallel/store.py) so the padded-vocab logits GEMMs see a whole [Vp, D] operand
        self.lm_head.weight._dpc_pad_rows = 64
        # execution state (not modules / not in the state_dict)
        object.__setattr__(self, "param_store", None)
        object.__setattr__(self, "stage", None)  # pipeline stage descriptor (None = whole model)
        # dropout: per-forward seeds = (dropout_seed_base << 32) | call counter
        self.dropout_seed_base = 0
        self._dropout_calls = 0
        object.__setattr__(self, "_seed_dev", None)  # device counter (next_dropout_seed)
        object.__setattr__(self, "_seed_dev_base", None)
        object.__setattr__(self, "_seed_snaps", {})  # host seed -> its device snapshot
        self.recompute = False  # per-layer activation recompute in the backward
        for i, layer in enumerate(self.decoder.layers):
            layer._layer_index = i

    # ------------------------------------------------------------------ dropout
    def next_dropout_seed(self) -> int:
        """Seed of the next training forward (each call advances the stream).

        On a GPU the seed also lives in device memory: a snapshot of the device counter
        (low word = forward count, high word = per-rank base) is taken and the counter is
        advanced with device ops, so a captured step (the HIP-graph "compile") replays with a
        new seed every time -- the kernels derive each site's key from the snapshot
        (``ops/dropout.py:DropSpec``).  Eager, both counters advance together and give the
        same masks as the host seed."""
        seed = ((self.dropout_seed_base & 0xFFFFFFFF) << 32) | (self._dropout_calls & 0xFFFFFFFF)
        self._dropout_calls += 1
        dev = next((q.device for q in self.parameters() if q.device.type != "meta"), None)
        if dev is not None and dev.type == "cuda":
            import torch

            def i32(v):
                v &= 0xFFFFFFFF
                return v - (1 << 32) if v >= (1 << 31) else v

            base = i32(self.dropout_seed_base)
            # (re)created on a new base or after the model moved to another device (model.to)
            if self._seed_dev is None or self._seed_dev_base != base or self._seed_dev.device != dev:
                self._seed_dev = torch.tensor([i32(seed), base], dtype=torch.int32, device=dev)
                self._seed_dev_base = base
            snap = self._seed_dev.clone()
            self._seed_dev[0:1].add_(1)  # (int32 wraps like the u32 word the kernels read)
            self._seed_snaps[seed] = snap
            while len(self._seed_snaps) > 256:  # (a pipeline step keeps at most M in flight)
                self._seed_snaps.pop(next(iter(self._seed_snaps)))
        return seed

    def dropout_specs(self, layer, seed, drawn: bool = False):
        """(attention-output, FFN-output) :class:`DropSpec` of ``layer`` for ``seed``.
        ``drawn``: the seed came from ``next_dropout_seed`` -- only then do the kernels read its
        device snapshot (after graph replays the device counter runs ahead of the host one, so
        an explicit ``dropout_seed`` equal to an old drawn value must keep its host key)."""
        from ..ops.dropout import DropSpec

        i = layer._layer_index
        snap = self._seed_snaps.get(seed) if drawn else None
        return (DropSpec.make(self.dropout, seed, 2 * i, snap),
                DropSpec.make(self.dropout, seed, 2 * i + 1, snap))

    # ------------------------------------------------------------------ structure
    def units(self):
        """Parameter units in forward order: the granularity of sharding / bucketing /
        pipeline partitioning (embeddings, one per decoder layer, head)."""
        out = [("embeddings", [self.embeddings])]
        out += [(f"decoder.layers.{i}", [l]) for i, l in enumerate(self.decoder.layers)]
        out.append(("head", [self.norm_out, self.lm_head]))
        return out

    def reference_forward(self, input_ids, position_ids, mask=None, dropout_seed=None):
        """The reference's math with plain torch modules (autograd does the backward).

        ``dropout_seed`` pins the dropout masks to those the fused path draws for that seed.
        """
        if dropout_seed is not None:
            for layer in self.decoder.layers:
                layer.attn.dropout.spec, layer.fc.dropout.spec = self.dropout_specs(layer, dropout_seed)
        try:
            x = self.embeddings(input_ids, position_ids)
            x = self.decoder(x, mask=mask)
            x = self.norm_out(x)
            return self.lm_head(x)
        finally:
            if dropout_seed is not None:
                for layer in self.decoder.layers:
                    layer.attn.dropout.spec = layer.fc.dropout.spec = None

    def forward(self, input_ids, position_ids, mask=None, targets=None, want_correct=False,
                dropout_seed=None, last_only=False):
        from .fused import fused_lm_forward

        return fused_lm_forward(self, input_ids, position_ids, mask, targets, want_correct, dropout_seed,
                                last_only)

    def new_kv_cache(self, batch_size: int, max_len: int):
        from .fused import KVCache, ensure_store

        return KVCache(self, batch_size, max_len, next(self.parameters()).device,
                       ensure_store(self).compute_dtype)

    def decode(self, input_ids, position_ids, cache):
        """Logits ``[N, 1, V]`` of the last of the new tokens, attending over ``cache`` (extended)."""
        from .fused import kv_decode_forward

        return kv_decode_forward(self, input_ids, position_ids, cache)

    def graph_decoder(self, cache):
        """HIP-graph one-token decode step over ``cache`` (None for a sharded store)."""
        from ..parallel.store import LocalStore
        from ..ops.attention import DECODE_MAX_S, decode_supported
        from .fused import GraphDecoder, ensure_store

        store = ensure_store(self)
        # the graphed step runs the HIP decode kernel, which reads the cache length on the
        # device; anything it does not take (an f32 store under --disable_amp, a head size it
        # does not handle) decodes eagerly instead -- the torch fallback reads the length on
        # the host, which a graph capture does not allow
        attn = self.decoder.layers[0].attn
        if (not isinstance(store, LocalStore) or cache.capacity > DECODE_MAX_S
                or store.compute_dtype != torch.bfloat16 or not decode_supported(attn.head_dim)):
            return None
        return GraphDecoder(self, cache)


PRESETS = {
    # reference default (argparse of every main-*.py)
    "ref": dict(dim=256, head_dim=32, heads=8, num_layers=8, sequence_length=256, activation="relu"),
    "gpt2-small": dict(dim=768, head_dim=64, heads=12, num_layers=12, sequence_length=1024, activation="gelu"),
    "gpt2-medium": dict(dim=1024, head_dim=64, heads=16, num_layers=24, sequence_length=1024, activation="gelu"),
    "gpt2-large": dict(dim=1280, head_dim=64, heads=20, num_layers=36, sequence_length=1024, activation="gelu"),
    "gpt2-xl": dict(dim=1600, head_dim=64, heads=25, num_layers=48, sequence_length=1024, activation="gelu"),
}
