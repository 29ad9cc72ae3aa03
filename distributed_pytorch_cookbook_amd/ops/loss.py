"""Fused softmax cross-entropy over the vocabulary (loss, dlogits, argmax accuracy).

Reference: ``F.cross_entropy(logits.view(-1, V), targets.view(-1), ignore_index=-100)``
(``/root/reference/main-single.py:95-96``) and the eval accuracy
``argmax(logits)[mask] == targets[mask]`` (``main-single.py:128-131``).

The HIP kernel makes one read pass (online max / sum-exp / argmax per row) and one
read-write pass that overwrites the bf16 logits with ``dlogits = (softmax - onehot) /
n_valid`` -- the [T, V] logits are never materialised in f32 and are read twice total.
``n_valid`` is a device scalar, so the step has no host synchronisation.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import _lib

IGNORE_INDEX = -100


def cross_entropy_rows(logits: torch.Tensor, targets: torch.Tensor, vocab: int, inv_count: torch.Tensor,
                       row_loss: torch.Tensor, row_correct: torch.Tensor | None = None,
                       write_grad: bool = True, ignore_index: int = IGNORE_INDEX) -> None:
    """HIP kernel on a block of rows: per-row loss (and argmax hit) into ``row_loss`` /
    ``row_correct``, dlogits = (softmax - onehot) * inv_count in place.  ``inv_count`` is the
    device scalar 1 / n_valid of the WHOLE batch, so a batch can be processed in row chunks
    (the chunked head keeps each chunk's logits resident in the Infinity Cache between the
    logits GEMM and this pass)."""
    T = logits.shape[0]
    if logits.stride(1) != 1 or logits.stride(0) % 8 or logits.data_ptr() % 16:
        raise ValueError("cross_entropy_rows: rows must be contiguous, 16-B aligned, ld % 8 == 0")
    tg = targets.reshape(-1).to(torch.int64).contiguous()
    args = _lib.CEArgs(
        logits=logits.data_ptr(), dlogits=logits.data_ptr(), targets=tg.data_ptr(),
        inv_count=inv_count.data_ptr(), row_loss=row_loss.data_ptr(), row_correct=_lib.ptr(row_correct),
        ld=logits.stride(0), T=T, V=vocab, write_grad=int(write_grad), ignore_index=ignore_index,
    )
    _lib.call("dpc_cross_entropy", args, logits.device)


def cross_entropy_fused(logits: torch.Tensor, targets: torch.Tensor, vocab: int,
                        write_grad: bool = True, want_correct: bool = False,
                        ignore_index: int = IGNORE_INDEX):
    """logits [T, ld >= vocab] (bf16 on HIP; padded columns ignored).

    Returns (loss_mean (0-dim f32), n_valid (0-dim f32), n_correct (0-dim f32) or None).
    If ``write_grad`` the logits buffer is overwritten IN PLACE with d(loss_mean)/d(logits)
    (padding columns zeroed).
    """
    T = logits.shape[0]
    tg = targets.reshape(-1)
    valid = tg != ignore_index
    n_valid = valid.sum().float()
    if not (logits.is_cuda and logits.dtype == torch.bfloat16):
        lv = logits[:, :vocab].float()
        loss_sum = F.cross_entropy(lv, tg, ignore_index=ignore_index, reduction="sum")
        correct = None
        if want_correct:
            correct = ((lv.argmax(-1) == tg) & valid).sum().float()
        if write_grad:
            p = torch.softmax(lv, dim=-1)
            safe = torch.where(valid, tg, torch.zeros_like(tg))
            p[torch.arange(T, device=lv.device), safe] -= 1.0
            p = p * (valid.float() / n_valid.clamp_min(1.0))[:, None]
            logits.zero_()
            logits[:, :vocab].copy_(p)
        return loss_sum / n_valid.clamp_min(1.0), n_valid, correct
    if logits.stride(1) != 1 or logits.stride(0) % 8 or logits.data_ptr() % 16:
        raise ValueError("cross_entropy_fused: rows must be contiguous, 16-B aligned, ld % 8 == 0")
    tg = tg.to(torch.int64).contiguous()
    inv = 1.0 / n_valid.clamp_min(1.0)
    row_loss = torch.empty(T, device=logits.device, dtype=torch.float32)
    row_correct = torch.empty(T, device=logits.device, dtype=torch.float32) if want_correct else None
    args = _lib.CEArgs(
        logits=logits.data_ptr(), dlogits=logits.data_ptr(), targets=tg.data_ptr(),
        inv_count=inv.data_ptr(), row_loss=row_loss.data_ptr(), row_correct=_lib.ptr(row_correct),
        ld=logits.stride(0), T=T, V=vocab, write_grad=int(write_grad), ignore_index=ignore_index,
    )
    _lib.call("dpc_cross_entropy", args, logits.device)
    loss = row_loss.sum() * inv
    return loss, n_valid, (row_correct.sum() if want_correct else None)
