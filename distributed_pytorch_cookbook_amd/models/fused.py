"""Fused execution of ``TransformerDecoderLM``: one autograd function per parameter unit.

Forward / backward of a decoder layer (reference ``models/gpt.py:108-135`` and the ops
it calls), as kernel calls on the bf16 compute weights of the parameter store:

  forward                                      backward (dx3 arrives f32)
  h1  = LN1(x)                 bf16            dz2 = dx3 * act'(z2) -> bf16, db2 += colsum
  qkv = h1 @ [Wq;Wk;Wv]^T      one GEMM        dW2 += dz2^T u ; dz1 = (dz2 @ W2) * act'(.)  (+db1 colsum)
  o   = flash_attn(qkv)        causal+pad      dW1 += dz1^T h2 ; dh2 = dz1 @ W1 (f32)
  x2  = x + o @ Wo^T + bo      epilogue        dx2 = dx3 + LN2'(dh2)      (in place)
  h2  = LN2(x2)                bf16            dYo = bf16(dx2), dbo += colsum ; dWo += dYo^T o
  u   = act(h2 @ W1^T + b1)    epilogue        do = dYo @ Wo ; dqkv = flash_attn_bwd
  x3  = x2 + act(u @ W2^T+b2)  epilogue, z2    dWqkv += dqkv^T h1 ; dh1 = dqkv @ Wqkv (f32)
                                               dx = dx2 + LN1'(dh1)       (in place)

Weight gradients are accumulated by the GEMM epilogues straight into the store's f32
gradient views (flat buffer), and each function reports unit boundaries to the store
(``pre/post_forward``, ``pre/post_backward``) -- that is where DDP launches bucket
all-reduces and FSDP all-gathers / reduce-scatters, overlapped with this compute.
Q, K, V weights are adjacent in the flat layout, so ``[Wq; Wk; Wv]`` is a view.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional

import torch

from ..ops.attention import DECODE_MAX_S, attention_bwd, attention_fwd, decode_attention
from ..ops.elementwise import bias_act_bwd
from ..ops.dropout import dropout_residual
from ..ops.embedding import embedding_bwd, embedding_fwd
from ..ops.gemm import (ACT_GELU, ACT_MUL, ACT_NONE, ACT_RELU, act_code, linear_dgrad, linear_fwd, linear_wgrad,
                        register_side_stream)
from ..ops.loss import cross_entropy_fused, cross_entropy_rows
from ..ops.norm import layernorm_bwd, layernorm_fwd

LN_EPS = 1e-5
# input gradients feeding a LayerNorm backward: bf16 (as autocast makes them in the
# reference) unless DPC_DH_F32=1
_DH_F32 = os.environ.get("DPC_DH_F32", "0") == "1"


def _dh_dtype(cdt):
    return torch.float32 if _DH_F32 else cdt


# The LM-head input gradient dX = dlogits @ W_lm has K = the padded vocabulary (50304) and an
# [T, D] output: at a small D it is a handful of 256 x 256 tiles (the reference CLI default model,
# D = 256 at T = 16320: 64 tiles for 256 CUs), and a bf16 output cannot be split along K (the
# split-K kernel sums f32 slabs).  Below half a chip of tiles the product is formed in f32, which
# the persistent kernel splits along K to fill the chip; the final LayerNorm backward reads f32 dy
# as it does under DPC_DH_F32.  DPC_HEAD_DGRAD_F32=0 / 1 forces either form.  (The same rule for
# the layers' QKV / FFN-up input gradients, K = 3 D / 4 D, measured 1.7 % slower on that model --
# too short a K to split: profiles/r6_final2/ref_default_ln_dgrad_negative.log.)
_HEAD_DGRAD_F32 = os.environ.get("DPC_HEAD_DGRAD_F32", "auto")


def _head_dgrad_dtype(T, D, cdt):
    if _HEAD_DGRAD_F32 in ("0", "1"):
        return torch.float32 if _HEAD_DGRAD_F32 == "1" else _dh_dtype(cdt)
    tiles = ((T + 255) // 256) * ((D + 255) // 256)
    return torch.float32 if tiles < 128 else _dh_dtype(cdt)


# rows per chunk of the logits GEMM + cross-entropy (0 = whole batch at once).  Off by
# default: on GPT-2 small (B=32) chunks of 1024 / 2048 / 4096 rows ran 751K / 757K / 762K
# tok/s against 775-781K unchunked -- the smaller logits GEMMs lose more than the
# cache-resident cross-entropy pass gains.
_HEAD_CHUNK = int(os.environ.get("DPC_HEAD_CHUNK", "0"))


def vocab_ld(vocab: int) -> int:
    """Row stride of the logits buffer: 64-element aligned (16-B chunks, MFMA tiles)."""
    return (vocab + 63) // 64 * 64


@dataclass
class LMOutput:
    loss: torch.Tensor
    n_valid: torch.Tensor
    n_correct: Optional[torch.Tensor] = None


def _qkv_weight(store, attn):
    wq, wk, wv = (store.weight(m.weight) for m in (attn.to_q, attn.to_k, attn.to_v))
    n = wq.shape[0]
    if (wk.data_ptr() == wq.data_ptr() + wq.numel() * wq.element_size()
            and wv.data_ptr() == wk.data_ptr() + wk.numel() * wk.element_size()):
        return wq.as_strided((3 * n, wq.shape[1]), (wq.shape[1], 1))  # adjacent in the flat buffer
    return torch.cat([wq, wk, wv], 0)


def _head_weight_padded(store, head, rows: int):
    """[rows, D] view of the head's compute weight including the zero rows the flat layout
    reserves after it (``_dpc_pad_rows``); the plain [V, D] view if there are none."""
    w = store.weight(head.weight)
    V, D = w.shape
    if rows == V or getattr(head.weight, "_dpc_pad_rows", 0) == 0 or w.stride() != (D, 1):
        return w
    end = w.storage_offset() + rows * D
    if end * w.element_size() > w.untyped_storage().nbytes():
        return w
    return w.as_strided((rows, D), (D, 1))


def _qkv_grad(store, attn):
    gq, gk, gv = (store.grad(m.weight) for m in (attn.to_q, attn.to_k, attn.to_v))
    n = gq.shape[0]
    if (gk.data_ptr() == gq.data_ptr() + gq.numel() * 4 and gv.data_ptr() == gk.data_ptr() + gk.numel() * 4):
        return gq.as_strided((3 * n, gq.shape[1]), (gq.shape[1], 1)), None
    buf = torch.zeros(3 * n, gq.shape[1], device=gq.device, dtype=torch.float32)
    return buf, (gq, gk, gv)


# ---- zero-bubble pipeline schedule (parallel/pipeline.py:schedule_zb): inside
# ``defer_weight_grads(buf)`` a backward runs only its input-gradient chain (B); every
# weight-gradient GEMM, the embedding scatter and the store's post_backward hook of each unit
# (which launches a DDP bucket once the unit's gradients are final) are appended to ``buf`` as
# closures, in issue order, for the engine to run later as the W pass.  The closures hold their
# operands (dY, X) alive; the other saved activations are released with the autograd graph.
_W_DEFER: Optional[list] = None


class defer_weight_grads:
    def __init__(self, buf: list):
        self.buf = buf
        self.prev = None

    def __enter__(self):
        global _W_DEFER
        self.prev, _W_DEFER = _W_DEFER, self.buf
        return self.buf

    def __exit__(self, *exc):
        global _W_DEFER
        _W_DEFER = self.prev
        return False


def _w(fn) -> None:
    """Run a weight-gradient step now, or queue it for the W pass."""
    if _W_DEFER is not None:
        _W_DEFER.append(fn)
    else:
        fn()


class _EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, ids, pos, mod, store, training):
        u = mod._unit_id
        store.pre_forward(u)
        x = embedding_fwd(ids, pos, store.weight(mod.input_embeddings.weight),
                          store.weight(mod.position_embeddings.weight))
        store.post_forward(u, training)
        ctx.save_for_backward(ids, pos)
        ctx.mod, ctx.store = mod, store
        return x

    @staticmethod
    def backward(ctx, dx):
        ids, pos = ctx.saved_tensors
        mod, store = ctx.mod, ctx.store
        u = mod._unit_id
        store.pre_backward(u, need_weights=False)
        dxc = dx.contiguous()

        def scatter():  # (a W-pass op: nothing upstream waits for it)
            embedding_bwd(dxc, ids, pos, store.grad(mod.input_embeddings.weight),
                          store.grad(mod.position_embeddings.weight))
            store.post_backward(u)

        _w(scatter)
        return None, None, None, None, None, None


# DPC_FUSE_OUT_LN=0: out-projection with the bias + residual GEMM epilogue and a separate LN2
_FUSE_OUT_LN = os.environ.get("DPC_FUSE_OUT_LN", "1") == "1"


def _layer_forward(x, mask, layer, store, N, S, act, training, drops, attend=None, pre=None, fuse_out=None):
    """Decoder-layer forward on the store's compute weights (no store hooks).

    Returns ``(x3, saved)``; ``saved`` holds what the backward needs when ``training``.
    ``attend(qkv) -> (o, lse)`` replaces the causal self-attention over these S tokens
    (the KV-cache decode attends over the cached keys instead).
    ``pre``: the previous layer's FFN output not yet added to the residual stream,
    ``(x2, z2, drop, act)`` -- x is then an unwritten buffer that LN1 fills with
    ``x2 + drop(act(z2))`` as it normalises (``_ResidualHandoff``).  ``fuse_out``: a
    ``_ResidualHandoff`` to leave this layer's own FFN output in, for the next layer's LN1
    (the returned x3 is then the buffer that LN1 will fill).
    """
    drop_attn, drop_ffn = drops
    attn, fc = layer.attn, layer.fc
    H, hd = attn.heads, attn.head_dim
    w = store.weight
    T, D = x.shape
    cdt = store.compute_dtype
    if pre is not None:  # the previous layer's down projection: residual add + act + dropout here
        x2p, z2p, dropp, actp = pre
        h1, mu1, rs1 = layernorm_fwd(x2p, w(layer.norm1.weight), w(layer.norm1.bias), LN_EPS, cdt,
                                     add=(z2p, None, dropp, actp), x_out=x)
    else:
        h1, mu1, rs1 = layernorm_fwd(x, w(layer.norm1.weight), w(layer.norm1.bias), LN_EPS, cdt)
    qkv = linear_fwd(h1, _qkv_weight(store, attn), out_dtype=cdt)
    o, lse = attention_fwd(qkv, N, S, H, hd, mask, causal=True) if attend is None else attend(qkv)
    if x.is_cuda and cdt == torch.bfloat16 and _FUSE_OUT_LN:
        # out-projection as a plain product (the hand-written v7 / v9 MFMA GEMM, bf16 out -- the
        # reference's autocast Linear output dtype) and its bias / dropout / residual add fused into LN2, which
        # writes the new f32 residual stream x2: the residual is read and written once,
        # instead of by a memory-bound GEMM epilogue and again by LN2
        yo = linear_fwd(o, w(attn.to_out.weight), out_dtype=cdt)
        x2 = torch.empty(T, D, device=x.device, dtype=torch.float32)
        h2, mu2, rs2 = layernorm_fwd(x, w(layer.norm2.weight), w(layer.norm2.bias), LN_EPS, cdt,
                                     add=(yo, w(attn.to_out.bias), drop_attn), x_out=x2)
    else:
        if drop_attn is None:
            x2 = linear_fwd(o, w(attn.to_out.weight), bias=w(attn.to_out.bias), residual=x,
                            out_dtype=torch.float32)
        else:
            x2 = linear_fwd(o, w(attn.to_out.weight), bias=w(attn.to_out.bias), out_dtype=torch.float32)
            dropout_residual(x2, x, drop_attn, out=x2)
        h2, mu2, rs2 = layernorm_fwd(x2, w(layer.norm2.weight), w(layer.norm2.bias), LN_EPS, cdt)
    F4 = w(fc.up_proj.weight).shape[0]
    # GELU: the up-projection's second output is GELU'(z1) (bf16), so the backward's input
    # gradient is dz1 = (dz2 @ W2) * g1 -- a plain multiply in its epilogue (ACT_MUL) instead of
    # the tanh-derivative math there; ReLU's act' comes from its own output (uact > 0)
    g1 = torch.empty(T, F4, device=x.device, dtype=cdt) if (training and act == ACT_GELU) else None
    uact = linear_fwd(h2, w(fc.up_proj.weight), bias=w(fc.up_proj.bias), act=act, aux_out=g1,
                      out_dtype=cdt, aux_deriv=g1 is not None)
    if fuse_out is not None:
        # x3 = x2 + drop(act(z2)) is formed by the NEXT layer's LN1 (one f32 read of x2 and one
        # write of x3 there, beside its own reads) instead of this GEMM's epilogue (f32 residual
        # read, f32 x3 + bf16 z2 writes under the MFMA tail: gemm7 EPI 9): the down projection
        # is a plain product with a bias, bf16 out -- z2 itself, kept for the backward
        z2 = linear_fwd(uact, w(fc.down_proj.weight), bias=w(fc.down_proj.bias), out_dtype=cdt)
        fuse_out.pending = (x2, z2, drop_ffn, act)
        x3 = torch.empty(T, D, device=x.device, dtype=torch.float32)
        saved = None
        if training:
            saved = (h1, mu1, rs1, qkv, o, lse, x2, h2, mu2, rs2, g1 if g1 is not None else uact, uact, z2)
        return x3, saved
    z2 = torch.empty(T, D, device=x.device, dtype=cdt) if training else None
    if drop_ffn is None:
        x3 = linear_fwd(uact, w(fc.down_proj.weight), bias=w(fc.down_proj.bias), act=act,
                        residual=x2, aux_out=z2, out_dtype=torch.float32)
    else:
        x3 = linear_fwd(uact, w(fc.down_proj.weight), bias=w(fc.down_proj.bias), act=act,
                        aux_out=z2, out_dtype=torch.float32)
        dropout_residual(x3, x2, drop_ffn, out=x3)
    saved = None
    if training:
        saved = (h1, mu1, rs1, qkv, o, lse, x2, h2, mu2, rs2, g1 if g1 is not None else uact, uact, z2)
    return x3, saved


class _FfnTail:
    """A layer's FFN down projection seen from the LayerNorm that consumes its output (the next
    layer's LN1, or the final norm).  The reference's FFN ends in ``drop(act(z2))`` added to the
    residual, so the first backward op of a layer is ``dz2 = bf16(dx3 * keep * act'(z2))`` plus
    the bias column sums -- one pass over the f32 residual gradient dx3 that the consumer's
    LayerNorm backward has just written.  The consumer does it in that pass instead
    (layernorm_bwd's gout / gz): it leaves dz2 here and adds the column sums straight into the
    bias gradient (a 1-D parameter: the stores keep those gradients valid for the whole backward,
    and no bucket holding it is reduced before the layer's own backward ends); the layer's own
    backward then starts from dz2.  Filled in the forward only when the layer keeps its
    activations (no recompute: z2 must exist when the consumer's backward runs)."""

    __slots__ = ("z2", "act", "drop", "dz2", "bias_grad", "fuse_next", "pending")

    def __init__(self, fuse_next: bool = False):
        self.z2 = self.act = self.drop = self.dz2 = self.bias_grad = None
        # forward: this layer's FFN output is added to the residual stream by the next layer's
        # LN1 (``pending`` = (x2, z2, drop, act) until it has been)
        self.fuse_next = fuse_next
        self.pending = None

    def consume(self, ln_bwd_kwargs, T, D, device, cdt):
        """Extend a LayerNorm backward call with this tail's fused consumer (if it has one)."""
        if self.z2 is None:
            return
        self.dz2 = torch.empty(T, D, device=device, dtype=cdt)
        ln_bwd_kwargs.update(gout=self.dz2, gsum=self.bias_grad(), drop=self.drop)
        if self.act != ACT_NONE:
            ln_bwd_kwargs.update(gz=self.z2, gact=self.act)
        self.z2 = None


# the fused consumer needs a bf16 operand on the GPU (the kernel's gout); off: DPC_FUSE_FFN_TAIL=0
_FUSE_TAIL = os.environ.get("DPC_FUSE_FFN_TAIL", "1") == "1"
# the FFN down projection's residual add / act / dropout in the next layer's LN1 forward (a plain
# bias GEMM then writes z2); off: DPC_FUSE_FFN_LN=0 (the gemm7 EPI 9 epilogue does it)
_FUSE_FFN_LN = os.environ.get("DPC_FUSE_FFN_LN", "1") == "1"


def _tail_ok(x, cdt):
    return _FUSE_TAIL and (cdt == torch.bfloat16 or not x.is_cuda)


class _LayerFn(torch.autograd.Function):
    """One decoder layer.  With ``recompute`` only the layer input is kept and the forward
    is re-run at the start of the backward (activation recompute: the saved activations of
    a layer drop from ~34 D bytes per token -- h1, qkv, o, x2, h2, u, z1, z2 -- to the 4 D
    bytes of its f32 input, for one extra forward)."""

    @staticmethod
    def forward(ctx, x, mask, layer, store, N, S, act, training, drops=(None, None), recompute=False,
                prev_tail=None, tail=None):
        u = layer._unit_id
        store.pre_forward(u)
        pre = None
        if prev_tail is not None and prev_tail.pending is not None:
            pre, prev_tail.pending = prev_tail.pending, None
        fuse = tail if (tail is not None and tail.fuse_next) else None
        x3, saved = _layer_forward(x, mask, layer, store, N, S, act, training and not recompute, drops,
                                   pre=pre, fuse_out=fuse)
        store.post_forward(u, training)
        if training:
            ctx.save_for_backward(x, mask, *(saved or ()))
            ctx.layer, ctx.store, ctx.dims, ctx.act = layer, store, (N, S), act
            ctx.drops, ctx.recompute = drops, recompute
            ctx.fused_out = fuse is not None  # (the recompute re-runs the same down-projection form)
            ctx.prev_tail, ctx.tail = prev_tail, tail
            if tail is not None and saved is not None and _tail_ok(x, store.compute_dtype):
                tail.z2, tail.act, tail.drop = saved[-1], act, drops[1]
                bias = layer.fc.down_proj.bias
                tail.bias_grad = lambda: store.grad(bias)
        return x3

    @staticmethod
    def backward(ctx, dx3):
        x, mask, *saved = ctx.saved_tensors
        layer, store, act = ctx.layer, ctx.store, ctx.act
        N, S = ctx.dims
        H, hd = layer.attn.heads, layer.attn.head_dim
        store.pre_backward(layer._unit_id)
        if ctx.recompute:
            _, saved = _layer_forward(x, mask, layer, store, N, S, act, True, ctx.drops,
                                      fuse_out=_FfnTail() if ctx.fused_out else None)
        dx = _layer_backward(dx3, x, mask, saved, layer, store, N, S, H, hd, act, ctx.drops,
                             ctx.prev_tail, ctx.tail)
        u = layer._unit_id
        _w(lambda: store.post_backward(u))  # (after the unit's deferred weight gradients)
        return dx, None, None, None, None, None, None, None, None, None, None, None


# Weight gradients of a layer run on a side HIP stream, concurrently with the input-gradient
# chain (bias/act backward -> dgrad -> LayerNorm backward -> attention backward) they do not
# feed: each wgrad waits for the main stream (its dY is ready), the main stream joins the side
# stream once at the end of the layer's backward, before the store's post_backward hook (DDP
# bucket all-reduce / FSDP reduce-scatter) reads the gradients.  Both run inside the HIP-graph
# capture as a fork / join.  Off by default (DPC_WGRAD_STREAM=1 turns it on): on one MI355X
# the GEMMs already fill the chip, and GPT-2 small B=64 measured 822.5 / 822.8K tok/s with
# the side stream against 825.2 / 824.2K without; FSDP GPT-2 XL 68.6K vs 68.8K
# (profiles/r1_v19_wgrad_stream_ab.txt).
_WGRAD_STREAM = os.environ.get("DPC_WGRAD_STREAM", "0") == "1"
_side_streams: dict = {}


class _SideWork:
    def __init__(self, device: torch.device):
        self.on = _WGRAD_STREAM and device.type == "cuda"
        self.stream = None
        if self.on:
            key = torch.cuda.current_stream(device).cuda_stream
            if key not in _side_streams:
                _side_streams[key] = torch.cuda.Stream(device=device)
                register_side_stream(_side_streams[key])
            self.stream = _side_streams[key]

    def run(self, fn, *tensors):
        if _W_DEFER is not None:  # zero-bubble schedule: the W pass runs it later
            _W_DEFER.append(fn)
            return
        if not self.on:
            fn()
            return
        self.stream.wait_stream(torch.cuda.current_stream(self.stream.device))
        with torch.cuda.stream(self.stream):
            fn()
        for t in tensors:  # temporaries freed by the main stream: not reused before the side reads
            t.record_stream(self.stream)

    def join(self):
        if self.on:
            torch.cuda.current_stream(self.stream.device).wait_stream(self.stream)


def _layer_backward(dx3, x, mask, saved, layer, store, N, S, H, hd, act, drops, prev_tail=None, tail=None):
    """Hand-written backward of ``_layer_forward``; weight grads go into the store.  ``tail``:
    this layer's _FfnTail (dz2 already formed by the consumer's LayerNorm backward);
    ``prev_tail``: the previous layer's, served by this layer's LN1 backward."""
    (h1, mu1, rs1, qkv, o, lse, x2, h2, mu2, rs2, zup, uact, z2) = saved
    attn, fc = layer.attn, layer.fc
    w, g = store.weight, store.grad
    cdt = store.compute_dtype
    drop_attn, drop_ffn = drops
    dx = dx3.contiguous()  # becomes dx2 then dx (in place)
    # FFN down projection: x3 = x2 + drop(act(z2)), z2 = u W2^T + b2
    side = _SideWork(dx.device)
    if tail is not None and tail.dz2 is not None:  # formed by the consumer's LayerNorm backward
        dz2 = tail.dz2  # (its bias column sums are already in the gradient)
        tail.dz2 = None
    else:
        dz2 = bias_act_bwd(dx, z2, act, g(fc.down_proj.bias), out_dtype=cdt, drop=drop_ffn)
    side.run(lambda: linear_wgrad(dz2, uact, out=g(fc.down_proj.weight)), dz2, uact)
    # up projection gradient with act' fused (relu' from its output; gelu'(z1) was stored by the
    # forward epilogue: a multiply)
    dz1 = linear_dgrad(dz2, w(fc.down_proj.weight), act_bwd=ACT_MUL if act == ACT_GELU else act, aux_in=zup,
                       out_dtype=cdt, colsum=g(fc.up_proj.bias))
    side.run(lambda: linear_wgrad(dz1, h2, out=g(fc.up_proj.weight)), dz1, h2)
    dh2 = linear_dgrad(dz1, w(fc.up_proj.weight), out_dtype=_dh_dtype(cdt))
    # LN2 backward with the attention output projection's bias/dropout backward fused in:
    # x2 = x + drop(o Wo^T + bo)  ->  dYo = bf16(dx2 * keep), dbo += colsum
    dyo = torch.empty(dx.shape, device=dx.device, dtype=cdt)
    layernorm_bwd(dh2, x2, mu2, rs2, w(layer.norm2.weight), dx, g(layer.norm2.weight),
                  g(layer.norm2.bias), gout=dyo, gsum=g(attn.to_out.bias), drop=drop_attn)
    side.run(lambda: linear_wgrad(dyo, o, out=g(attn.to_out.weight)), dyo, o)
    do = linear_dgrad(dyo, w(attn.to_out.weight), out_dtype=cdt)
    dqkv = attention_bwd(do, qkv, o, lse, N, S, H, hd, mask, causal=True)
    gqkv, split = _qkv_grad(store, attn)

    def qkv_wgrad():
        linear_wgrad(dqkv, h1, out=gqkv)
        if split is not None:
            n = split[0].shape[0]
            for i, gi in enumerate(split):
                gi.add_(gqkv[i * n:(i + 1) * n])

    side.run(qkv_wgrad, dqkv, h1, gqkv)
    dh1 = linear_dgrad(dqkv, _qkv_weight(store, attn), out_dtype=_dh_dtype(cdt))
    kw = {}
    if prev_tail is not None:  # the previous layer's down-projection bias / act / dropout backward
        prev_tail.consume(kw, x.shape[0], x.shape[1], x.device, cdt)
    layernorm_bwd(dh1, x, mu1, rs1, w(layer.norm1.weight), dx, g(layer.norm1.weight),
                  g(layer.norm1.bias), **kw)
    side.join()
    return dx


def _ln_in(x, pending, gamma, beta, cdt):
    """LayerNorm of x -- or, with the previous layer's FFN output still pending (x an unwritten
    buffer), of x2 + drop(act(z2)), written into x on the way (``_FfnTail.pending``)."""
    if pending is None:
        return layernorm_fwd(x, gamma, beta, LN_EPS, cdt)
    x2p, z2p, dropp, actp = pending
    return layernorm_fwd(x2p, gamma, beta, LN_EPS, cdt, add=(z2p, None, dropp, actp), x_out=x)


_unit_ln = {}


def materialize_pending(x, tail) -> None:
    """Form a run's output x3 = x2 + drop(act(z2)) in place when no LayerNorm consumes it in the
    same pass (a pipeline stage boundary, the last-row decode head): through the same fused
    LayerNorm kernel (its normalised output discarded), so x3 has the same bits whichever way it is
    formed -- a layer's position in a run never changes the math."""
    if tail is None or tail.pending is None:
        return
    pending, tail.pending = tail.pending, None
    D = x.shape[1]
    key = (x.device, D)
    if key not in _unit_ln:
        _unit_ln[key] = (torch.ones(D, device=x.device), torch.zeros(D, device=x.device))
    g, b = _unit_ln[key]
    with torch.no_grad():
        _ln_in(x, pending, g, b, pending[1].dtype)


class _HeadFn(torch.autograd.Function):
    """norm_out -> lm_head -> fused cross-entropy (reference gpt.py:229-231 + main-*.py loss)."""

    @staticmethod
    def forward(ctx, x, targets, norm, head, store, unit, training, want_correct, prev_tail=None):
        store.pre_forward(unit)
        w = store.weight
        cdt = store.compute_dtype
        V = w(head.weight).shape[0]
        T = x.shape[0]
        pending = None
        if prev_tail is not None and prev_tail.pending is not None:  # the last layer's FFN output
            pending, prev_tail.pending = prev_tail.pending, None
        hf, mu, rs = _ln_in(x, pending, w(norm.weight), w(norm.bias), cdt)
        ld = vocab_ld(V) if x.is_cuda else V
        buf = torch.empty(T, ld, device=x.device, dtype=cdt)
        # padded columns come out 0 (B rows >= V are the layout's zero rows / read as 0)
        wpad = _head_weight_padded(store, head, ld)
        chunk = _HEAD_CHUNK if (x.is_cuda and cdt == torch.bfloat16) else 0
        if chunk and T > chunk:
            # row chunks: each chunk's bf16 logits (chunk x Vp x 2 B) are still in the 256 MB
            # Infinity Cache when the cross-entropy pass reads them back
            tg = targets.reshape(-1)
            n_valid = (tg != -100).sum().float()
            inv = 1.0 / n_valid.clamp_min(1.0)
            row_loss = torch.empty(T, device=x.device, dtype=torch.float32)
            row_corr = torch.empty(T, device=x.device, dtype=torch.float32) if want_correct else None
            for c0 in range(0, T, chunk):
                c1 = min(T, c0 + chunk)
                linear_fwd(hf[c0:c1], wpad, out=buf[c0:c1])
                cross_entropy_rows(buf[c0:c1], tg[c0:c1], V, inv, row_loss[c0:c1],
                                   None if row_corr is None else row_corr[c0:c1], write_grad=training)
            loss = row_loss.sum() * inv
            n_correct = row_corr.sum() if want_correct else None
        else:
            linear_fwd(hf, wpad, out=buf)
            loss, n_valid, n_correct = cross_entropy_fused(buf, targets, V, write_grad=training,
                                                           want_correct=want_correct)
        store.post_forward(unit, training)
        if training:
            ctx.save_for_backward(x, hf, mu, rs, buf)
            ctx.mods, ctx.store, ctx.unit, ctx.V = (norm, head), store, unit, V
            ctx.prev_tail = prev_tail
        ctx.mark_non_differentiable(n_valid)
        if n_correct is None:
            n_correct = torch.zeros((), device=x.device)
        ctx.mark_non_differentiable(n_correct)
        return loss, n_valid, n_correct

    @staticmethod
    def backward(ctx, dloss, _dn, _dc):
        x, hf, mu, rs, dlogits = ctx.saved_tensors
        (norm, head), store, unit, V = ctx.mods, ctx.store, ctx.unit, ctx.V
        store.pre_backward(unit)
        w, g = store.weight, store.grad
        dl = dlogits[:, :V]
        scale = dloss.reshape(()).float().contiguous()
        _w(lambda: linear_wgrad(dl, hf, out=g(head.weight), alpha_t=scale))
        # K = padded vocab: the CE kernel zeroed dlogits' pad columns, W_lm rows >= V read as 0
        dhf = linear_dgrad(dlogits, _head_weight_padded(store, head, dlogits.shape[1]),
                           out_dtype=_head_dgrad_dtype(x.shape[0], x.shape[1], store.compute_dtype),
                           alpha_t=scale)
        dx = torch.empty_like(x)  # (written, not accumulated: dx_set)
        kw = {}
        if ctx.prev_tail is not None:  # the last layer's down-projection bias / act / dropout backward
            ctx.prev_tail.consume(kw, x.shape[0], x.shape[1], x.device, store.compute_dtype)
        layernorm_bwd(dhf, x, mu, rs, w(norm.weight), dx, g(norm.weight), g(norm.bias), dx_set=True, **kw)
        _w(lambda: store.post_backward(unit))
        return dx, None, None, None, None, None, None, None, None


def head_logits(model, x, store, tail=None):
    """Inference head: logits [T, V] (view of a row-padded buffer), no loss.  ``tail``: the last
    layer's, whose FFN output the final norm adds to the residual stream (x then unwritten)."""
    w = store.weight
    unit = model._head_unit_id
    store.pre_forward(unit)
    V = w(model.lm_head.weight).shape[0]
    pending = None
    if tail is not None and tail.pending is not None:
        pending, tail.pending = tail.pending, None
    hf, _, _ = _ln_in(x, pending, w(model.norm_out.weight), w(model.norm_out.bias), store.compute_dtype)
    ld = vocab_ld(V) if x.is_cuda else V
    buf = torch.empty(x.shape[0], ld, device=x.device, dtype=store.compute_dtype)
    linear_fwd(hf, w(model.lm_head.weight), out=buf)
    store.post_forward(unit, False)
    return buf[:, :V]


def ensure_store(model):
    store = model.param_store
    if store is None:
        from ..parallel.store import LocalStore

        dev = next(model.parameters()).device
        store = LocalStore(model, dev)
    return store


def run_embeddings(model, store, input_ids, position_ids, training):
    anchor = store.anchor if training else store.anchor.detach()
    return _EmbedFn.apply(anchor, input_ids.reshape(-1), position_ids.reshape(-1),
                          model.embeddings, store, training)


def run_layers(model, store, x, mask, N, S, layers, training, dropout_seed=None, head_next=False):
    """``training``: keep activations for the backward.  Dropout follows the module mode
    (``model.train()`` / ``model.eval()``) like ``nn.Dropout``.  ``head_next``: the model's final
    norm consumes the output in this pass (``run_head`` / ``head_logits`` with the returned
    tensor's ``_dpc_tail``), so the last layer's residual add is left to it as every other
    layer's is left to the next layer's LN1; otherwise the output is formed here."""
    act = act_code(model.activation)
    use_drop = model.training and model.dropout > 0
    if use_drop and dropout_seed is None:
        dropout_seed = model.next_dropout_seed()
        drawn = True
    else:
        drawn = False
    recompute = bool(getattr(model, "recompute", False)) and training
    prev = None
    fuse_ok = _FUSE_FFN_LN and (store.compute_dtype == torch.bfloat16 or not x.is_cuda)
    for i, layer in enumerate(layers):
        drops = model.dropout_specs(layer, dropout_seed, drawn) if use_drop else (None, None)
        # every layer hands its FFN output to the next LayerNorm (the last one to the final norm,
        # or to materialize_pending below): one formula for x3 whatever the layer's position
        tail = _FfnTail(fuse_next=fuse_ok)
        x = _LayerFn.apply(x, mask, layer, store, N, S, act, training, drops, recompute, prev, tail)
        prev = tail
    if prev is not None:
        if head_next:
            x._dpc_tail = prev  # (the final norm consumes the last layer's output -- forward and backward)
        else:
            materialize_pending(x, prev)
            if training:
                x._dpc_tail = prev  # (backward only: the head's LN bwd, if any, takes dz2)
    return x


def run_head(model, store, x, targets, training, want_correct):
    return _HeadFn.apply(x, targets.reshape(-1), model.norm_out, model.lm_head, store,
                         model._head_unit_id, training, want_correct, getattr(x, "_dpc_tail", None))


def last_rows(x, N, S):
    """[N*S, D] -> [N, D]: the last position of every sequence (all a greedy decode step needs)."""
    return x.view(N, S, -1)[:, -1].contiguous()


def fused_lm_forward(model, input_ids, position_ids, mask=None, targets=None, want_correct=False,
                     dropout_seed=None, last_only=False):
    store = ensure_store(model)
    N, S = input_ids.shape
    training = torch.is_grad_enabled()
    if mask is not None:
        mask = mask.to(device=input_ids.device, dtype=torch.bool).contiguous()
    x = run_embeddings(model, store, input_ids, position_ids, training)
    x = run_layers(model, store, x, mask, N, S, model.decoder.layers, training, dropout_seed,
                   head_next=not (targets is None and last_only))
    if targets is None:
        if last_only:  # decode: LM head on the last position only ([N, 1, V]; T x fewer FLOPs)
            return head_logits(model, last_rows(x, N, S), store).reshape(N, 1, -1)
        return head_logits(model, x, store, getattr(x, "_dpc_tail", None)).reshape(N, S, -1)
    loss, n_valid, n_correct = run_head(model, store, x, targets, training, want_correct)
    return LMOutput(loss, n_valid, n_correct if want_correct else None)


class KVCache:
    """Keys / values of every layer for the tokens decoded so far: ``[N, S_max, H*hd]`` each
    in the compute dtype (GPT-2 XL at S_max = 1024: 2 x 48 x 1024 x 1600 x 2 B = 315 MB per
    sequence)."""

    def __init__(self, model, N, S_max, device, dtype):
        self.k, self.v = [], []
        for layer in model.decoder.layers:
            E = layer.attn.heads * layer.attn.head_dim
            # zeroed: the graphed step reads the whole capacity (masked, but 0 * NaN = NaN)
            self.k.append(torch.zeros(N, S_max, E, device=device, dtype=dtype))
            self.v.append(torch.zeros(N, S_max, E, device=device, dtype=dtype))
        self.len = 0
        self.capacity = S_max
        self.len_t = torch.zeros(1, device=device, dtype=torch.int64)  # device copy for the graph


def _cached_attention(qkv, cache, li, N, n, H, hd):
    """Append the n new tokens' K/V to layer li's cache and attend to every cached key.

    Prefill (empty cache) is the flash-attention kernel over the n tokens; a decode step is
    n queries against ``start + n`` keys -- a memory-bound read of the cache (GEMV-shaped,
    no tiles to fill), done as two batched products in f32."""
    E = H * hd
    start = cache.len
    L = start + n
    q3 = qkv.view(N, n, 3, E)
    cache.k[li][:, start:L] = q3[:, :, 1]
    cache.v[li][:, start:L] = q3[:, :, 2]
    if start == 0:
        return attention_fwd(qkv, N, n, H, hd, None, causal=True)
    q = q3[:, :, 0].float().reshape(N, n, H, hd).transpose(1, 2)             # [N, H, n, hd]
    k = cache.k[li][:, :L].float().reshape(N, L, H, hd).transpose(1, 2)     # [N, H, L, hd]
    v = cache.v[li][:, :L].float().reshape(N, L, H, hd).transpose(1, 2)
    sc = (q @ k.transpose(-1, -2)) * (1.0 / math.sqrt(hd))                  # [N, H, n, L]
    if n > 1:  # causal inside the new block: query i sees keys < start + i + 1
        qi = torch.arange(n, device=qkv.device)[:, None] + start
        sc = sc.masked_fill(torch.arange(L, device=qkv.device)[None, :] > qi, float("-inf"))
    o = torch.softmax(sc, -1) @ v                                            # [N, H, n, hd]
    return o.transpose(1, 2).reshape(N * n, E).to(qkv.dtype), None


def kv_decode_forward(model, input_ids, position_ids, cache):
    """Incremental forward for greedy decoding: runs only the new tokens (the whole prompt
    on the first call, then one token per call) through the layers, extends ``cache`` and
    returns the logits of the last new token, ``[N, 1, V]``.  Same kernels as the training
    forward (LayerNorm, QKV / FFN GEMMs with fused epilogues, the LM head); the reference
    recomputes the whole sequence for every token (``/root/reference/utils.py:57-65``)."""
    store = ensure_store(model)
    N, n = input_ids.shape
    if cache.len + n > cache.capacity:
        raise ValueError(f"KV cache full ({cache.len} + {n} > {cache.capacity})")
    act = act_code(model.activation)
    x = run_embeddings(model, store, input_ids, position_ids, False)
    for li, layer in enumerate(model.decoder.layers):
        H, hd = layer.attn.heads, layer.attn.head_dim
        u = layer._unit_id
        store.pre_forward(u)
        x, _ = _layer_forward(x, None, layer, store, N, n, act, False, (None, None),
                              attend=lambda qkv, li=li, H=H, hd=hd: _cached_attention(qkv, cache, li, N, n, H, hd))
        store.post_forward(u, False)
    cache.len += n
    cache.len_t.fill_(cache.len)
    return head_logits(model, last_rows(x, N, n), store).reshape(N, 1, -1)


def _static_attention(qkv, cache, li, N, H, hd):
    """One query per sequence against the cache, the new key / value appended at the
    device-side length by the decode kernel: no shape depends on the length, so the step
    can be graphed."""
    return decode_attention(qkv, cache.k[li], cache.v[li], cache.len_t, H, hd), None


class GraphDecoder:
    """The one-token decode step (embedding, every layer, LM head, cache append) captured
    once as a HIP graph and replayed per token: a GPT-2 decode step is a few hundred small
    launches, so eager decoding is launch-bound (measured in ``bench/generate.py``).  Needs
    a non-sharded parameter store (single GPU / DDP); FSDP decodes eagerly."""

    def __init__(self, model, cache):
        self.model, self.cache = model, cache
        self.store = ensure_store(model)
        N = cache.k[0].shape[0]
        self.tok = torch.zeros(N, 1, device=cache.len_t.device, dtype=torch.int64)
        self.graph = None
        self.out = None

    def _step(self):
        model, store, cache = self.model, self.store, self.cache
        N = self.tok.shape[0]
        act = act_code(model.activation)
        x = run_embeddings(model, store, self.tok, cache.len_t.expand(N, 1), False)
        for li, layer in enumerate(model.decoder.layers):
            H, hd = layer.attn.heads, layer.attn.head_dim
            x, _ = _layer_forward(x, None, layer, store, N, 1, act, False, (None, None),
                                  attend=lambda qkv, li=li, H=H, hd=hd: _static_attention(qkv, cache, li, N, H, hd))
        cache.len_t.add_(1)
        return head_logits(model, x, store).reshape(N, 1, -1)

    def step(self, tok):
        """Append ``tok`` [N, 1] at the cache's current length; logits [N, 1, V] (a view of the
        graph's output buffer, overwritten by the next step)."""
        cache = self.cache
        if cache.len + 1 > cache.capacity:
            raise ValueError(f"KV cache full ({cache.len} + 1 > {cache.capacity})")
        self.tok.copy_(tok)
        if self.graph is None:
            self._step()                 # eager warm-up (lazy library init), then undo it
            cache.len_t.sub_(1)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.out = self._step()
            self.graph = g
        self.graph.replay()
        cache.len += 1
        return self.out
