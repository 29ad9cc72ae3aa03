"""Token + learned-position embedding (gather-add) and its scatter-add backward.

Reference: ``/root/reference/models/gpt.py:169-185`` (``Embeddings``: two nn.Embedding
lookups summed; the f32 result is the residual stream).
"""
from __future__ import annotations

import os

import torch

from . import _lib


def embedding_fwd(ids: torch.Tensor, pos: torch.Tensor, tok: torch.Tensor, ptab: torch.Tensor,
                  out: torch.Tensor | None = None) -> torch.Tensor:
    """ids, pos int64 [T]; tables [V, D], [P, D] (f32 or bf16) -> f32 [T, D]."""
    T = ids.numel()
    D = tok.shape[1]
    if not tok.is_cuda:
        x = tok[ids.reshape(-1)].float() + ptab[pos.reshape(-1)].float()
        if out is not None:
            out.copy_(x)
            return out
        return x
    ids = ids.reshape(-1).to(torch.int64).contiguous()
    pos = pos.reshape(-1).to(torch.int64).contiguous()
    if tok.dtype != ptab.dtype or tok.dtype not in (torch.float32, torch.bfloat16):
        raise ValueError("embedding_fwd: tables must share dtype f32/bf16")
    if not (tok.is_contiguous() and ptab.is_contiguous()) or D % 4:
        raise ValueError("embedding_fwd: contiguous tables with D % 4 == 0 required")
    if out is None:
        out = torch.empty(T, D, device=tok.device, dtype=torch.float32)
    args = _lib.EmbArgs(
        ids=ids.data_ptr(), pos=pos.data_ptr(), tok=tok.data_ptr(), ptab=ptab.data_ptr(),
        out=out.data_ptr(), T=T, D=D, V=tok.shape[0], P=ptab.shape[0],
        table_bf16=int(tok.dtype == torch.bfloat16),
    )
    _lib.call("dpc_embedding_fwd", args, tok.device)
    return out


# Deterministic backward (csrc/embed_bwd.hip): a stable radix sort of (id, row) pairs and one
# writer per table row, summing its rows in row order -- bitwise reproducible, no float atomics.
# DPC_EMB_ATOMIC=1 selects the atomic scatter (misc.hip) instead (A/B only).
_ATOMIC = os.environ.get("DPC_EMB_ATOMIC", "0") == "1"
_ws: dict = {}


def _workspace(device, T: int, D: int):
    """Sort workspace for T rows, per device, grown on demand outside any graph capture (a
    captured step keeps the buffer it was recorded with)."""
    need = int(_lib.lib().dpc_embedding_bwd_ws(int(T), int(D)))
    t = _ws.get(device.index)
    if t is None or t.numel() < need:
        if torch.cuda.is_current_stream_capturing():
            return None
        t = torch.empty(max(need, 256), dtype=torch.uint8, device=device)
        _ws[device.index] = t
    return t


def embedding_bwd(dout: torch.Tensor, ids: torch.Tensor, pos: torch.Tensor,
                  dtok: torch.Tensor | None, dpos: torch.Tensor | None) -> None:
    """dtok[ids] += dout; dpos[pos] += dout (f32 grads)."""
    if not dout.is_cuda:
        ids = ids.reshape(-1)
        pos = pos.reshape(-1)
        if dtok is not None:
            dtok.index_add_(0, ids, dout.to(dtok.dtype))
        if dpos is not None:
            dpos.index_add_(0, pos, dout.to(dpos.dtype))
        return
    ids = ids.reshape(-1).to(torch.int64).contiguous()
    pos = pos.reshape(-1).to(torch.int64).contiguous()
    dout = dout.contiguous()
    ref = dtok if dtok is not None else dpos
    args = _lib.EmbArgs(
        ids=ids.data_ptr(), pos=pos.data_ptr(), dout=dout.data_ptr(), dtok=_lib.ptr(dtok),
        dpos=_lib.ptr(dpos), T=ids.numel(), D=dout.shape[1],
        V=dtok.shape[0] if dtok is not None else 2**31 - 1,
        P=dpos.shape[0] if dpos is not None else 2**31 - 1,
    )
    if dtok is not None and dtok.dtype != torch.float32 or dpos is not None and dpos.dtype != torch.float32:
        raise ValueError("embedding_bwd: f32 gradient tables required")
    D = dout.shape[1]
    ws = None if (_ATOMIC or D % 4 or D > 2048) else _workspace(ref.device, ids.numel(), D)
    if ws is not None:
        sargs = _lib.EmbBwdArgs(
            ids=ids.data_ptr(), pos=pos.data_ptr(), dout=dout.data_ptr(), dtok=_lib.ptr(dtok),
            dpos=_lib.ptr(dpos), ws=ws.data_ptr(), ws_bytes=ws.numel(), T=ids.numel(), D=D,
            V=args.V, P=args.P)
        _lib.call("dpc_embedding_bwd_sorted", sargs, ref.device)
        return
    _lib.call("dpc_embedding_bwd", args, ref.device)
