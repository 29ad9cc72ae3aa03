"""LayerNorm forward/backward over the f32 residual stream.

Reference: ``nn.LayerNorm`` at ``/root/reference/models/gpt.py:119,122,217`` (eps 1e-5,
elementwise affine).  Forward: f32 x -> normalised y (bf16 on the HIP path, feeding the
next GEMM) + per-row (mean, rstd).  Backward: ``dx += LN'(dy)`` accumulated in place
into the residual-gradient buffer, with dgamma / dbeta accumulated into f32 grads.
"""
from __future__ import annotations

import torch

from . import _lib
from .dropout import keep_mask
from .gemm import act_grad_ref


def _use_hip(x: torch.Tensor, y_dtype: torch.dtype, add=None) -> bool:
    """bf16 y (the AMP path) or f32 y (--disable_amp); the fused residual add takes a bf16 y."""
    return (x.is_cuda and y_dtype in (torch.bfloat16, torch.float32)
            and (add is None or add[0].dtype == torch.bfloat16))


def layernorm_fwd(x: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float = 1e-5,
                  out_dtype: torch.dtype = torch.bfloat16, out: torch.Tensor | None = None,
                  add=None, x_out: torch.Tensor | None = None):
    """x [T, D] f32 -> (y [T, D] out_dtype, mean [T], rstd [T]).

    ``add=(y, bias, drop[, act])`` fuses the residual add of the projection that feeds this
    LayerNorm: the row normalised is ``xs = x + drop(act(y + bias))`` (y the plain GEMM output,
    bf16 on the HIP path; drop a ``dropout.Drop`` or None; act an activation code, default none
    -- the FFN down projection's GELU / ReLU), and ``xs`` is written to ``x_out`` (f32 [T, D]) --
    the new residual stream, read once and written once instead of the GEMM epilogue writing it
    and this kernel reading it back."""
    T, D = x.shape
    if add is not None and x_out is None:
        raise ValueError("layernorm_fwd: add= needs x_out")
    if not _use_hip(x, out_dtype, add):
        if add is not None:
            y_add, b_add, drop, act = (tuple(add) + (0,))[:4]
            a = y_add.float() + (b_add.float() if b_add is not None else 0.0)
            if act:
                from .gemm import act_fwd_ref

                a = act_fwd_ref(a, act)
            if drop is not None:
                a = a * keep_mask(drop, T, D, x.device)
            x_out.copy_(x.float() + a)
            x = x_out
        xf = x.float()
        mean = xf.mean(-1)
        var = xf.var(-1, unbiased=False)
        rstd = torch.rsqrt(var + eps)
        y = (xf - mean[:, None]) * rstd[:, None] * gamma.float() + beta.float()
        if out is not None:
            out.copy_(y)
            y = out
        else:
            y = y.to(out_dtype)
        return y, mean, rstd
    if x.dtype != torch.float32 or x.stride(1) != 1 or D % 4 or D > 2048:
        raise ValueError("layernorm_fwd: need f32 x with contiguous rows, D % 4 == 0, D <= 2048")
    if out is None:
        out = torch.empty(T, D, device=x.device, dtype=out_dtype)
    mean = torch.empty(T, device=x.device, dtype=torch.float32)
    rstd = torch.empty(T, device=x.device, dtype=torch.float32)
    args = _lib.LNArgs(
        x=x.data_ptr(), gamma=gamma.data_ptr(), beta=beta.data_ptr(), y=out.data_ptr(),
        mean=mean.data_ptr(), rstd=rstd.data_ptr(), ldx=x.stride(0), ldy=out.stride(0),
        T=T, D=D, eps=float(eps), y_f32=int(out.dtype == torch.float32),
    )
    if add is not None:
        y_add, b_add, drop, act = (tuple(add) + (0,))[:4]
        if (y_add.dtype != torch.bfloat16 or y_add.stride(1) != 1 or y_add.stride(0) % 4
                or x_out.dtype != torch.float32 or x_out.stride(1) != 1 or x_out.stride(0) % 4
                or tuple(y_add.shape) != (T, D) or tuple(x_out.shape) != (T, D)
                or (b_add is not None and (b_add.dtype != torch.float32 or not b_add.is_contiguous()))):
            raise ValueError("layernorm_fwd: add= needs bf16 y [T, D], f32 bias [D], f32 x_out [T, D]")
        args.add_y, args.add_bias, args.x_out = y_add.data_ptr(), _lib.ptr(b_add), x_out.data_ptr()
        args.ld_add, args.ld_xout = y_add.stride(0), x_out.stride(0)
        args.add_act = int(act or 0)
        if drop is not None:
            if T * D >= 2 ** 32:
                raise ValueError("layernorm_fwd: dropout needs T * D < 2^32")
            args.drop_key, args.drop_thresh, args.drop_scale = drop.key, drop.thresh, drop.scale
            args.drop_seed, args.drop_site = drop.seed_ptr(), drop.site
    _lib.call("dpc_layernorm_fwd", args, x.device)
    return out, mean, rstd


def layernorm_bwd(dy: torch.Tensor, x: torch.Tensor, mean: torch.Tensor, rstd: torch.Tensor,
                  gamma: torch.Tensor, dx: torch.Tensor, dgamma: torch.Tensor, dbeta: torch.Tensor,
                  gout: torch.Tensor | None = None, gsum: torch.Tensor | None = None,
                  drop=None, gz: torch.Tensor | None = None, gact=None, dx_set: bool = False):
    """dx += LN'(dy); dgamma += sum dy*xhat; dbeta += sum dy.  x, dx f32 [T, D]; dy f32 or
    bf16 (the input gradient of the Linear that consumed the LayerNorm's output -- bf16 under
    the reference's autocast too).

    Optional fused consumer of the updated dx (the backward of the bias + dropout of the
    projection whose output fed this LayerNorm's residual): ``gout = dx * keep`` (bf16,
    the next GEMM's operand) and ``gsum += colsum(dx * keep)`` (that projection's bias
    gradient), saving a separate pass over the f32 dx.  With ``gz`` (bf16 [T, D]) and ``gact``
    the projection's output went through an activation first (the reference's FFN applies it
    after the down projection too): ``gout = dx * keep * act'(gz)``.  ``dx_set``: dx = LN'(dy),
    dx's old contents neither read nor needed (the final norm's backward: no zero fill).
    """
    T, D = x.shape
    if not (x.is_cuda and dy.dtype in (torch.float32, torch.bfloat16) and gamma.dtype == torch.float32
            and (gout is None or gout.dtype == torch.bfloat16)):
        xh = (x.float() - mean[:, None]) * rstd[:, None]
        dyf = dy.float()
        dg = dyf * gamma.float()
        s1 = dg.mean(-1, keepdim=True)
        s2 = (dg * xh).mean(-1, keepdim=True)
        g_ln = rstd[:, None] * (dg - s1 - xh * s2)
        if dx_set:
            dx.copy_(g_ln)
        else:
            dx.add_(g_ln)
        dgamma.add_((dyf * xh).sum(0))
        dbeta.add_(dyf.sum(0))
        if gout is not None:
            g = dx if drop is None else dx * keep_mask(drop, T, D, dx.device)
            if gz is not None:
                g = g * act_grad_ref(gz.float(), gact)
            gout.copy_(g)
            if gsum is not None:
                gsum.add_(g.sum(0))
        return dx
    for t, nm in ((x, "x"), (dx, "dx")):
        if t.dtype != torch.float32 or t.stride(1) != 1:
            raise ValueError(f"layernorm_bwd: {nm} must be f32 with contiguous rows")
    if dy.stride(1) != 1 or (dy.dtype == torch.bfloat16 and (dy.stride(0) % 4 or dy.data_ptr() % 8)):
        raise ValueError("layernorm_bwd: dy must have contiguous (8-B aligned for bf16) rows")
    args = _lib.LNArgs(
        x=x.data_ptr(), gamma=gamma.data_ptr(), mean=mean.data_ptr(), rstd=rstd.data_ptr(),
        dy=dy.data_ptr(), dx=dx.data_ptr(), dgamma=dgamma.data_ptr(), dbeta=dbeta.data_ptr(),
        ldx=x.stride(0), lddy=dy.stride(0), lddx=dx.stride(0), T=T, D=D, eps=0.0,
        dy_bf16=int(dy.dtype == torch.bfloat16), dx_set=int(dx_set),
    )
    if gout is not None:
        if gout.dtype != torch.bfloat16 or gout.stride(1) != 1 or gout.stride(0) % 4 or D % 4:
            raise ValueError("layernorm_bwd: gout must be bf16 with 8-B aligned contiguous rows")
        args.gout, args.gsum, args.ld_gout = gout.data_ptr(), _lib.ptr(gsum), gout.stride(0)
        if gz is not None:
            if (gz.dtype != torch.bfloat16 or gz.shape != x.shape or gz.stride(1) != 1 or gz.stride(0) % 4
                    or gz.data_ptr() % 8):
                raise ValueError("layernorm_bwd: gz must be bf16 [T, D] with 8-B aligned contiguous rows")
            args.gz, args.ld_gz, args.gact = gz.data_ptr(), gz.stride(0), int(gact)
        if drop is not None:
            if T * D >= 2 ** 32:
                raise ValueError("layernorm_bwd: dropout needs T * D < 2^32")
            args.drop_key, args.drop_thresh, args.drop_scale = drop.key, drop.thresh, drop.scale
            args.drop_seed, args.drop_site = drop.seed_ptr(), drop.site
    _lib.call("dpc_layernorm_bwd", args, x.device)
    return dx
