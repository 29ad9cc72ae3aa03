"""Batch preparation and greedy generation (reference ``/root/reference/utils.py``).

``prepare_batch`` keeps the reference contract -- shift by one for next-token targets,
targets equal to ``pad_id`` become -100, position ids 0..S-2, ``mask = ~attention_mask``
(True = padded key) -- with two changes: an all-valid batch gets ``mask=None`` (decided
on the host before the copy, so no device sync; an all-False padding mask is a no-op)
and the position ids are built on the device instead of being copied.

``generate`` is the reference's greedy argmax loop (``utils.py:42-91``): full
recompute per token, stop at EOS, decode with ``skip_special_tokens``.  ``model`` is any
callable ``model(input_ids=..., position_ids=...) -> logits [1, s, V]`` (an LM or a
parallel engine's forward), so FSDP / pipeline engines run it on every rank.
"""
from __future__ import annotations

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
def generate(model, prompt: str, tokenizer, device, max_new_tokens: int = 20) -> str:
    batch = tokenizer([prompt], truncation=True, max_length=256, return_tensors="pt")
    input_ids = batch["input_ids"].to(device)
    # the learned position table bounds the context: slide a window past it
    max_pos = getattr(model, "max_position_embeddings", None) or 1 << 30
    for _ in range(max_new_tokens):
        ctx = input_ids[:, -max_pos:]
        s = ctx.shape[1]
        position_ids = torch.arange(s, device=device).unsqueeze(0)
        logits = model(input_ids=ctx, position_ids=position_ids)
        new_token = int(logits[0, -1].argmax(dim=-1))
        if new_token == tokenizer.eos_token_id:
            break
        input_ids = torch.cat([input_ids, torch.tensor([[new_token]], dtype=input_ids.dtype, device=device)], 1)
    return tokenizer.decode(input_ids[0].tolist(), skip_special_tokens=True)
