"""Bias + activation backward, f32 -> bf16 casts.

``bias_act_bwd`` turns an f32 upstream gradient into the bf16 GEMM operand
``dz = dy * act'(z)`` and accumulates the bias gradient ``db += colsum(dz)`` in the same
pass (reference: the autograd of ``nn.Linear`` bias + ``F.relu`` at
``/root/reference/models/gpt.py:33-41,102``).
"""
from __future__ import annotations

import torch

from . import _lib
from .dropout import DropSpec, keep_mask
from .gemm import act_code, act_grad_ref


def bias_act_bwd(dy: torch.Tensor, z: torch.Tensor | None, act, db: torch.Tensor | None,
                 out: torch.Tensor | None = None, out_dtype=torch.bfloat16,
                 drop: DropSpec | None = None) -> torch.Tensor:
    """``dz = dy * keep * act'(z)``; ``drop`` is the forward's dropout of this site."""
    act = act_code(act)
    T, N = dy.shape
    if not (dy.is_cuda and out_dtype == torch.bfloat16):
        g = dy.float()
        if drop is not None:
            g = g * keep_mask(drop, T, N, dy.device)
        if act:
            g = g * act_grad_ref(z, act)
        if db is not None:
            db.add_(g.sum(0))
        if out is not None:
            out.copy_(g)
            return out
        return g.to(out_dtype)
    if (dy.dtype != torch.float32 or dy.stride(1) != 1 or N % 4 or dy.stride(0) % 4
            or dy.data_ptr() % 16):
        raise ValueError("bias_act_bwd: f32 dy with 16-B aligned contiguous rows, N % 4 == 0")
    if act and (z is None or z.dtype != torch.bfloat16 or z.stride(1) != 1 or z.stride(0) % 4
                or z.data_ptr() % 8):
        raise ValueError("bias_act_bwd: bf16 pre-activation z required")
    if out is None:
        out = torch.empty(T, N, device=dy.device, dtype=torch.bfloat16)
    args = _lib.BiasActArgs(
        dy=dy.data_ptr(), z=_lib.ptr(z), dz=out.data_ptr(), db=_lib.ptr(db),
        lddy=dy.stride(0), ldz=z.stride(0) if z is not None else 0, lddz=out.stride(0),
        T=T, N=N, act=act,
    )
    if drop is not None:
        if T * N >= 2 ** 32:
            raise ValueError("bias_act_bwd: dropout needs T * N < 2^32")
        args.drop_key, args.drop_thresh, args.drop_scale = drop.key, drop.thresh, drop.scale
        args.drop_seed, args.drop_site = drop.seed_ptr(), drop.site
    _lib.call("dpc_bias_act_bwd", args, dy.device)
    return out


def cast_f32_bf16(src: torch.Tensor, dst: torch.Tensor) -> torch.Tensor:
    """Flat f32 -> bf16 copy (contiguous, numel % 4 == 0 on the HIP path)."""
    if not src.is_cuda or src.numel() % 4:
        dst.copy_(src)
        return dst
    assert src.is_contiguous() and dst.is_contiguous() and dst.dtype == torch.bfloat16
    args = _lib.CastArgs(src=src.data_ptr(), dst=dst.data_ptr(), n=src.numel())
    _lib.call("dpc_cast_f32_bf16", args, src.device)
    return dst
