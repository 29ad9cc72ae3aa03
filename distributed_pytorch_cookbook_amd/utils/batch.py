"""Batch preparation and greedy generation (reference ``/root/reference/utils.py``).

``prepare_batch`` keeps the reference contract -- shift by one for next-token targets,
targets equal to ``pad_id`` become -100, position ids 0..S-2, ``mask = ~attention_mask``
(True = padded key) -- with two changes: an all-valid batch gets ``mask=None`` (decided
on the host before the copy, so no device sync; an all-False padding mask is a no-op)
and the position ids are built on the device instead of being copied.

``generate`` is the reference's greedy argmax loop (``utils.py:42-91``): full
recompute per token, stop at EOS, decode with ``skip_special_tokens``; the LM head runs
on the last position only (``last_only``) where the model supports it, and a model with
``decode`` (``TransformerDecoderLM``) runs a KV-cache decode instead while the context fits.  ``model`` is any
callable ``model(input_ids=..., position_ids=...) -> logits [1, s, V]`` (an LM or a
parallel engine's forward), so FSDP / pipeline engines run it on every rank.
"""
from __future__ import annotations

import inspect

import torch


def prepare_batch(batch, pad_id: int, device):
    input_ids = batch["input_ids"]
    attention_mask = batch["attention_mask"][:, :-1]
    S = input_ids.shape[1]
    inputs, targets = input_ids[:, :-1].clone(), input_ids[:, 1:].clone()
    targets[targets == pad_id] = -100
    has_pad = not bool(attention_mask.all()) if attention_mask.device.type == "cpu" else True
    device = torch.device(device)
    nb = device.type == "cuda"
    position_ids = torch.arange(S - 1, device=device).unsqueeze(0).expand(inputs.shape[0], -1)
    out = dict(
        input_ids=inputs.to(device, non_blocking=nb),
        position_ids=position_ids,
        mask=(~attention_mask.to(dtype=torch.bool)).to(device, non_blocking=nb) if has_pad else None,
    )
    return out, targets.to(device, non_blocking=nb)


@torch.inference_mode()
def generate(model, prompt: str, tokenizer, device, max_new_tokens: int = 20, use_cache: bool = True) -> str:
    batch = tokenizer([prompt], truncation=True, max_length=256, return_tensors="pt")
    input_ids = batch["input_ids"].to(device)
    # the learned position table bounds the context: slide a window past it
    max_pos = getattr(model, "max_position_embeddings", None) or 1 << 30
    # only the last position's logits are used: skip the [T, V] head GEMM where the model can
    # (the reference computes every position's logits, utils.py:57-65)
    try:
        fwd = model.forward if isinstance(model, torch.nn.Module) else model
        last_only = "last_only" in inspect.signature(fwd).parameters
    except (TypeError, ValueError):
        last_only = False
    if use_cache and hasattr(model, "decode") and input_ids.shape[1] + max_new_tokens <= max_pos:
        return _generate_cached(model, input_ids, tokenizer, device, max_new_tokens)
    for _ in range(max_new_tokens):
        ctx = input_ids[:, -max_pos:]
        s = ctx.shape[1]
        position_ids = torch.arange(s, device=device).unsqueeze(0)
        if last_only:
            logits = model(input_ids=ctx, position_ids=position_ids, last_only=True)
        else:
            logits = model(input_ids=ctx, position_ids=position_ids)
        new_token = int(logits[0, -1].argmax(dim=-1))
        if new_token == tokenizer.eos_token_id:
            break
        input_ids = torch.cat([input_ids, torch.tensor([[new_token]], dtype=input_ids.dtype, device=device)], 1)
    return tokenizer.decode(input_ids[0].tolist(), skip_special_tokens=True)


def _generate_cached(model, input_ids, tokenizer, device, max_new_tokens):
    """KV-cache greedy decode: one prefill of the prompt, then one token per forward (same
    tokens as the full-recompute loop while the context fits the position table)."""
    cache = model.new_kv_cache(1, input_ids.shape[1] + max_new_tokens)
    s = input_ids.shape[1]
    logits = model.decode(input_ids, torch.arange(s, device=device).unsqueeze(0), cache)
    out = input_ids[0].tolist()
    step = None
    if device.type == "cuda" and hasattr(model, "graph_decoder"):
        step = model.graph_decoder(cache)  # None if the store is sharded (FSDP)
    for i in range(max_new_tokens):
        new_token = int(logits[0, -1].argmax(dim=-1))
        if new_token == tokenizer.eos_token_id:
            break
        out.append(new_token)
        if i + 1 == max_new_tokens:
            break
        tok = torch.tensor([[new_token]], dtype=input_ids.dtype, device=device)
        if step is not None:
            logits = step.step(tok)
        else:
            logits = model.decode(tok, torch.full((1, 1), len(out) - 1, device=device, dtype=torch.long), cache)
    return tokenizer.decode(out, skip_special_tokens=True)
