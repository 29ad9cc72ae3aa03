"""Causal self-attention core (softmax(q k^T * scale + masks) v) on the fused QKV buffer.

Semantics follow ``/root/reference/models/gpt.py:68-105``: causal mask (key j > query i
is excluded), optional key-padding mask (``True`` = padded key, excluded), softmax in
f32, output heads merged back to ``[T, H*hd]``.  One deliberate difference: a query row
whose every key is masked yields 0 here (the reference's finfo.min / -1e9 arithmetic
yields an ill-defined average); such rows only occur for all-padding sequences.

HIP path (bf16, head_dim 32, 64 or 128 natively): ``dpc_attn_fwd`` / ``dpc_attn_bwd`` flash
kernels (``csrc/attention.hip``) -- O(S) memory, f32 log-sum-exp saved for the backward.
f32 operands (``--disable_amp``) run ``dpc_attn_fwd_f32`` / ``dpc_attn_bwd_f32``
(``csrc/attention_f32.hip``, f32 matrix cores), also O(S).
head_dim 32 is the reference default config (``/root/reference/main-single.py:160``); other
head sizes up to 128 are zero-padded to the next kernel size on the way in (16 -> 32, 48 -> 64,
96 -> 128).  The reference's ``SelfAttention`` takes any ``--head_dim``
(``/root/reference/models/gpt.py:44-66``): sizes above 128 run the reference math on the
device (O(S^2) memory, correct but slow) rather than refusing.
CPU / fp32 path: the same math with torch ops (test oracle).
"""
from __future__ import annotations

import math

import torch

from . import _lib

HD_KERNELS = (32, 64, 128)
HD_KERNEL = 128  # the largest


def kernel_head_dim(head_dim: int) -> int | None:
    """The kernel size a head of ``head_dim`` runs at (itself for 32 / 64 / 128, else padded
    up); None above the largest kernel (the device then runs the reference math)."""
    for k in HD_KERNELS:
        if head_dim <= k:
            return k
    return None


def _use_hip(t: torch.Tensor, head_dim: int | None = None) -> bool:
    """bf16 -> csrc/attention.hip; f32 (--disable_amp) -> csrc/attention_f32.hip; head sizes
    past the largest kernel -> the reference math (on whatever device ``t`` is on)."""
    if head_dim is not None and kernel_head_dim(head_dim) is None:
        return False
    return t.is_cuda and t.dtype in (torch.bfloat16, torch.float32)


def _suffix(t: torch.Tensor) -> str:
    return "_f32" if t.dtype == torch.float32 else ""


def _check_span(t: torch.Tensor, S: int, *lds: int) -> None:
    """The bf16 kernels address one sequence's rows with 32-bit offsets (attention.hip:rows_rsrc):
    (S + 256) rows of every strided operand must span < 4 GiB."""
    if t.dtype != torch.float32 and (S + 256) * max(lds) * t.element_size() >= 0xFFFFFFFF:
        raise ValueError(f"attention: one sequence's rows span >= 4 GiB (S={S}, row strides {lds}); "
                         "split the sequence or run the reference path")


def split_qkv(qkv: torch.Tensor, heads: int, head_dim: int):
    """Views q, k, v [T, H*hd] out of the fused [T, 3*H*hd] projection."""
    hd = heads * head_dim
    return qkv[:, :hd], qkv[:, hd:2 * hd], qkv[:, 2 * hd:]


def attention_ref(qkv, N, S, heads, head_dim, pad_mask=None, causal=True, scale=None):
    """Reference math; returns (o [T, H*hd] in qkv.dtype, lse [N*H, S] f32)."""
    scale = 1.0 / math.sqrt(head_dim) if scale is None else scale
    q, k, v = split_qkv(qkv, heads, head_dim)
    q = q.float().reshape(N, S, heads, head_dim).transpose(1, 2)
    k = k.float().reshape(N, S, heads, head_dim).transpose(1, 2)
    v = v.float().reshape(N, S, heads, head_dim).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) * scale
    allowed = torch.ones(S, S, dtype=torch.bool, device=qkv.device)
    if causal:
        allowed = torch.tril(allowed)
    allowed = allowed.expand(N, 1, S, S)
    if pad_mask is not None:
        allowed = allowed & ~pad_mask.bool()[:, None, None, :]
    s = s.masked_fill(~allowed, float("-inf"))
    m = s.amax(-1, keepdim=True)
    m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    e = torch.exp(s - m)
    l = e.sum(-1, keepdim=True)
    p = torch.where(l > 0, e / l.clamp_min(1e-30), torch.zeros_like(e))
    o = (p @ v).transpose(1, 2).reshape(N * S, heads * head_dim)
    lse = torch.where(l > 0, m + torch.log(l.clamp_min(1e-30)), torch.full_like(l, float("inf")))
    return o.to(qkv.dtype), lse.reshape(N * heads, S)


def _pad_heads(x: torch.Tensor, T: int, heads: int, head_dim: int, kd: int) -> torch.Tensor:
    """[T, H*hd] (strided view ok) -> contiguous [T, H*kd] with zero padding."""
    out = torch.zeros(T, heads, kd, device=x.device, dtype=x.dtype)
    out[:, :, :head_dim] = x.reshape(T, heads, head_dim)
    return out.reshape(T, heads * kd)


def attention_fwd(qkv: torch.Tensor, N: int, S: int, heads: int, head_dim: int,
                  pad_mask: torch.Tensor | None = None, causal: bool = True,
                  out: torch.Tensor | None = None):
    """qkv [T = N*S, 3*H*hd] -> (o [T, H*hd], lse [N*H, S] f32)."""
    T = N * S
    if not _use_hip(qkv, head_dim):
        o, lse = attention_ref(qkv, N, S, heads, head_dim, pad_mask, causal)
        if out is not None:
            out.copy_(o)
            o = out
        return o, lse
    scale = 1.0 / math.sqrt(head_dim)
    kd = kernel_head_dim(head_dim)
    if head_dim != kd:
        q, k, v = split_qkv(qkv, heads, head_dim)
        qkv_p = torch.cat([_pad_heads(t, T, heads, head_dim, kd) for t in (q, k, v)], dim=1)
        o_p, lse = _attn_fwd_hip(qkv_p, N, S, heads, kd, pad_mask, causal, scale, None)
        o = o_p.reshape(T, heads, kd)[:, :, :head_dim].reshape(T, heads * head_dim)
        if out is not None:
            out.copy_(o)
            o = out
        return o.contiguous() if out is None else o, lse
    return _attn_fwd_hip(qkv, N, S, heads, kd, pad_mask, causal, scale, out)


def _check(t, T, cols, name, dtype=torch.bfloat16):
    if t.shape[0] != T or t.stride(1) != 1 or t.dtype != dtype:
        raise ValueError(f"attention: bad {name} {tuple(t.shape)} {t.stride()} {t.dtype}")
    if t.data_ptr() % 16 or t.stride(0) % (16 // t.element_size()) or t.shape[1] < cols:
        raise ValueError(f"attention: {name} must be 16-B aligned with 16-B aligned rows")


def _attn_fwd_hip(qkv, N, S, heads, kd, pad_mask, causal, scale, out):
    T = N * S
    hd = heads * kd
    dt = qkv.dtype
    _check(qkv, T, 3 * hd, "qkv", dt)
    if out is None:
        out = torch.empty(T, hd, device=qkv.device, dtype=dt)
    _check(out, T, hd, "out", dt)
    lse = torch.empty(N * heads, S, device=qkv.device, dtype=torch.float32)
    pad = None
    if pad_mask is not None:
        pad = pad_mask.to(torch.uint8).contiguous()
        assert pad.shape == (N, S)
    q, k, v = split_qkv(qkv, heads, kd)
    args = _lib.AttnArgs(
        q=q.data_ptr(), k=k.data_ptr(), v=v.data_ptr(), o=out.data_ptr(), lse=lse.data_ptr(),
        pad=_lib.ptr(pad), ld_qkv=qkv.stride(0), ld_o=out.stride(0), ld_dqkv=0,
        N=N, S=S, H=heads, scale=float(scale), causal=int(causal), hd=kd,
    )
    _check_span(qkv, S, qkv.stride(0), out.stride(0))
    _lib.call("dpc_attn_fwd" + _suffix(qkv), args, qkv.device)
    return out, lse


def attention_bwd(dout: torch.Tensor, qkv: torch.Tensor, o: torch.Tensor, lse: torch.Tensor,
                  N: int, S: int, heads: int, head_dim: int,
                  pad_mask: torch.Tensor | None = None, causal: bool = True,
                  dqkv: torch.Tensor | None = None) -> torch.Tensor:
    """Gradient w.r.t. the fused qkv buffer: returns dqkv [T, 3*H*hd] (qkv dtype)."""
    T = N * S
    if not _use_hip(qkv, head_dim):
        with torch.enable_grad():
            x = qkv.detach().float().requires_grad_(True)
            o_ref, _ = attention_ref(x, N, S, heads, head_dim, pad_mask, causal)
            (g,) = torch.autograd.grad(o_ref, x, dout.float())
        if dqkv is not None:
            dqkv.copy_(g)
            return dqkv
        return g.to(qkv.dtype)
    scale = 1.0 / math.sqrt(head_dim)
    kd = kernel_head_dim(head_dim)
    if head_dim != kd:
        q, k, v = split_qkv(qkv, heads, head_dim)
        qkv_p = torch.cat([_pad_heads(t, T, heads, head_dim, kd) for t in (q, k, v)], dim=1)
        o_p = _pad_heads(o, T, heads, head_dim, kd)
        do_p = _pad_heads(dout, T, heads, head_dim, kd)
        g_p = _attn_bwd_hip(do_p, qkv_p, o_p, lse, N, S, heads, kd, pad_mask, causal, scale, None)
        g = g_p.reshape(T, 3, heads, kd)[..., :head_dim].reshape(T, 3 * heads * head_dim)
        if dqkv is not None:
            dqkv.copy_(g)
            return dqkv
        return g.contiguous()
    return _attn_bwd_hip(dout, qkv, o, lse, N, S, heads, kd, pad_mask, causal, scale, dqkv)


def _attn_bwd_hip(dout, qkv, o, lse, N, S, heads, kd, pad_mask, causal, scale, dqkv):
    T = N * S
    hd = heads * kd
    dt = qkv.dtype
    dout = dout.to(dt)
    _check(qkv, T, 3 * hd, "qkv", dt)
    _check(o, T, hd, "o", dt)
    _check(dout, T, hd, "dout", dt)
    if o.stride(0) != dout.stride(0):
        dout = dout.contiguous()
        o = o.contiguous()
        if o.stride(0) != dout.stride(0):
            raise ValueError("attention_bwd: o and dout need equal row strides")
    if dqkv is None:
        dqkv = torch.empty(T, 3 * hd, device=qkv.device, dtype=dt)
    _check(dqkv, T, 3 * hd, "dqkv", dt)
    # [delta | lse in log2 units] rows (attn_bwd_pre_kernel writes both)
    delta = torch.empty(2, N * heads, S, device=qkv.device, dtype=torch.float32)
    pad = None
    if pad_mask is not None:
        pad = pad_mask.to(torch.uint8).contiguous()
    q, k, v = split_qkv(qkv, heads, kd)
    dq, dk, dv = split_qkv(dqkv, heads, kd)
    args = _lib.AttnArgs(
        q=q.data_ptr(), k=k.data_ptr(), v=v.data_ptr(), o=o.data_ptr(), lse=lse.data_ptr(),
        pad=_lib.ptr(pad), dout=dout.data_ptr(), dq=dq.data_ptr(), dk=dk.data_ptr(),
        dv=dv.data_ptr(), delta=delta.data_ptr(),
        ld_qkv=qkv.stride(0), ld_o=o.stride(0), ld_dqkv=dqkv.stride(0),
        N=N, S=S, H=heads, scale=float(scale), causal=int(causal), hd=kd,
    )
    _check_span(qkv, S, qkv.stride(0), o.stride(0))
    _lib.call("dpc_attn_bwd" + _suffix(qkv), args, qkv.device)
    return dqkv


DECODE_MAX_S = 16384  # csrc/decode.hip: LDS score buffer


def decode_supported(head_dim: int) -> bool:
    """Head sizes the decode kernel takes (16-B chunks of a row, at most one per thread)."""
    return head_dim > 0 and head_dim % 8 == 0 and head_dim <= 256


def decode_attention(qkv, kc, vc, length, heads, head_dim, scale=None):
    """One new token per sequence against a KV cache: appends its key / value at
    ``length`` (device int64 [1], cached tokens so far) and returns o [N, H*hd].

    qkv [N, 3*H*hd]; kc, vc [N, S_max, H*hd].  HIP path: ``dpc_decode_attn``
    (``csrc/decode.hip``); reads the length on the device, so it can be graph-captured.
    """
    scale = 1.0 / math.sqrt(head_dim) if scale is None else scale
    N, E = qkv.shape[0], heads * head_dim
    Smax = kc.shape[1]
    if not (qkv.is_cuda and qkv.dtype == torch.bfloat16):
        pos = int(length)
        q, k, v = split_qkv(qkv, heads, head_dim)
        kc[:, pos] = k
        vc[:, pos] = v
        qf = q.float().reshape(N, heads, 1, head_dim)
        kf = kc[:, :pos + 1].float().reshape(N, pos + 1, heads, head_dim).transpose(1, 2)
        vf = vc[:, :pos + 1].float().reshape(N, pos + 1, heads, head_dim).transpose(1, 2)
        p = torch.softmax((qf @ kf.transpose(-1, -2)) * scale, -1)
        return (p @ vf).reshape(N, E).to(qkv.dtype)
    if (qkv.stride(1) != 1 or kc.shape != (N, Smax, E) or vc.shape != kc.shape or not kc.is_contiguous()
            or not vc.is_contiguous() or kc.dtype != torch.bfloat16 or vc.dtype != torch.bfloat16
            or not decode_supported(head_dim) or Smax > DECODE_MAX_S
            or qkv.stride(0) % 8 or qkv.data_ptr() % 16 or length.dtype != torch.int64):
        raise ValueError("decode_attention: unsupported layout")
    o = torch.empty(N, E, device=qkv.device, dtype=torch.bfloat16)
    args = _lib.DecodeAttnArgs(qkv=qkv.data_ptr(), kc=kc.data_ptr(), vc=vc.data_ptr(), o=o.data_ptr(),
                               len=length.data_ptr(), ldqkv=qkv.stride(0), ldo=E, N=N, H=heads,
                               hd=head_dim, Smax=Smax, scale=scale)
    _lib.call("dpc_decode_attn", args, qkv.device)
    return o
