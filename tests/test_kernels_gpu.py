"""Numerics of every HIP kernel against a plain PyTorch f32 reference of the same op."""
import math

import pytest
import torch

from distributed_pytorch_cookbook_amd.ops import _lib
from distributed_pytorch_cookbook_amd.ops.attention import attention_bwd, attention_fwd, attention_ref
from distributed_pytorch_cookbook_amd.ops.elementwise import bias_act_bwd
from distributed_pytorch_cookbook_amd.ops.embedding import embedding_bwd, embedding_fwd
from distributed_pytorch_cookbook_amd.ops.gemm import _gemm_ref, gemm
from distributed_pytorch_cookbook_amd.ops.loss import cross_entropy_fused
from distributed_pytorch_cookbook_amd.ops.norm import layernorm_bwd, layernorm_fwd
from distributed_pytorch_cookbook_amd.ops.optim import FlatAdamW

pytestmark = pytest.mark.gpu
dev = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("a_kmaj,b_kmaj", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (200, 300, 136), (1023, 768, 768), (64, 50257, 64)])
def test_gemm_layouts(a_kmaj, b_kmaj, M, N, K):
    torch.manual_seed(0)
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    # pad the contiguous extent of mn-major operands to a multiple of 8 (as the model does)
    def store(x, kmaj):
        if kmaj:
            return x
        r, c = x.shape  # logical [mn, K] -> stored [K, mn_pad]
        buf = torch.zeros(c, (r + 7) // 8 * 8, device=dev, dtype=x.dtype)
        buf[:, :r] = x.t()
        return buf[:, :r]
    A, B = store(a, a_kmaj), store(b, b_kmaj)
    out = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out_dtype=torch.float32)
    ref = a.float() @ b.float().t()
    assert rel_err(out, ref) < 2e-3


@pytest.mark.parametrize("impl", [1, 2, 3, 4, 10])
@pytest.mark.parametrize("a_kmaj,b_kmaj", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (200, 296, 192), (1023, 768, 768), (77, 1000, 1023),
                                   (130, 136, 4160), (600, 520, 4160)])
def test_gemm_impls_with_epilogue(impl, a_kmaj, b_kmaj, M, N, K):
    torch.manual_seed(11)
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()

    def store(x, kmaj):
        r, c = x.shape
        if kmaj:  # rows padded to a multiple of 8 elements (16-B aligned row starts)
            buf = torch.zeros(r, (c + 7) // 8 * 8, device=dev, dtype=x.dtype)
            buf[:, :c] = x
            return buf[:, :c]
        buf = torch.zeros(c, (r + 7) // 8 * 8, device=dev, dtype=x.dtype)
        buf[:, :r] = x.t()
        return buf[:, :r]

    A, B = store(a, a_kmaj), store(b, b_kmaj)
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    z = torch.randn(M, N, device=dev).bfloat16()
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=dev)
    _lib.set_gemm_impl(impl)
    try:
        out = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, bias=bias, act=2, act_bwd=1, aux_in=z,
                   aux_out=aux, residual=res, colsum=cs, out_dtype=torch.float32)
        acc0 = torch.randn(M, N, device=dev)
        acc = acc0.clone()
        gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=acc, accumulate=True)
        ob = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj)  # bf16 out
        # act' without a residual: the aux operand rides the epilogue's prefetch slot
        cs2 = torch.zeros(N, device=dev)
        od = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, act_bwd=2, aux_in=z, colsum=cs2)
    finally:
        _lib.set_gemm_impl(-1)
    od_r = torch.empty(M, N, device=dev)
    cs2_r = torch.zeros(N, device=dev)
    _gemm_ref(a, b, True, True, od_r, None, 0, 2, z, None, None, 1.0, None, False, cs2_r)
    assert rel_err(od, od_r) < 1e-2
    assert rel_err(cs2, cs2_r) < 2e-3
    ref_out = torch.empty(M, N, device=dev)
    aux_r = torch.empty_like(aux)
    cs_r = torch.zeros(N, device=dev)
    _gemm_ref(a, b, True, True, ref_out, bias, 2, 1, z, aux_r, res, 1.0, None, False, cs_r)
    assert rel_err(out, ref_out) < 2e-3
    assert rel_err(aux, aux_r) < 1e-2
    assert rel_err(cs, cs_r) < 2e-3
    assert rel_err(acc - acc0, a.float() @ b.float().t()) < 2e-3
    assert rel_err(ob, a.float() @ b.float().t()) < 1e-2


def _store(x, kmaj):
    """Operand storage as the model lays it out: k-major rows (or mn-major columns) padded
    to a multiple of 8 elements."""
    r, c = x.shape
    if kmaj:
        buf = torch.zeros(r, (c + 7) // 8 * 8, device=dev, dtype=x.dtype)
        buf[:, :c] = x
        return buf[:, :c]
    buf = torch.zeros(c, (r + 7) // 8 * 8, device=dev, dtype=x.dtype)
    buf[:, :r] = x.t()
    return buf[:, :r]


@pytest.mark.parametrize("impl", [16, 17, 19, 20, 21, 22, 25, 26])
@pytest.mark.parametrize("a_kmaj,b_kmaj", [(True, True), (True, False), (False, False), (False, True)])
@pytest.mark.parametrize("M,N,K", [(300, 264, 128), (1023, 768, 768), (4096, 4352, 256), (513, 2304, 1536),
                                   (300, 264, 96), (257, 520, 1000)])
def test_gemm_v7_v8_v9(impl, a_kmaj, b_kmaj, M, N, K):
    """The 256x256 kernels on the shapes they serve: ragged M, N % 8 == 0, K % 64 == 0, and
    (4096 x 4352: 272 tiles) more tiles than CUs, so a persistent v7 workgroup streams two
    tiles through one ring -- plain bf16 / f32 outputs, accumulate and every fused epilogue.
    22 / 25: v7 with paired / split DMA issue; 26: v9 (64-deep stages) for the plain products it
    takes (K % 64 == 0), v7 for the rest; 16 / 19 / 20 / 22 also run v9 on plain nt products."""
    torch.manual_seed(3)
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    A, B = _store(a, a_kmaj), _store(b, b_kmaj)
    ref = a.float() @ b.float().t()
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    z = torch.randn(M, N, device=dev).bfloat16()
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=dev)
    acc0 = torch.randn(M, N, device=dev)
    acc = acc0.clone()
    _lib.set_gemm_impl(impl)
    try:
        ob = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj)
        of = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out_dtype=torch.float32, alpha=0.5)
        gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=acc, accumulate=True)
        out = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, bias=bias, act=2, act_bwd=1, aux_in=z,
                   aux_out=aux, residual=res, colsum=cs, out_dtype=torch.float32)
        cs2 = torch.zeros(N, device=dev)
        od = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, act_bwd=2, aux_in=z, colsum=cs2)
        og = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, bias=bias, act=2, aux_out=torch.empty_like(aux))
    finally:
        _lib.set_gemm_impl(-1)
    assert rel_err(ob, ref) < 1e-2
    assert rel_err(of, 0.5 * ref) < 2e-3
    assert rel_err(acc - acc0, ref) < 2e-3
    ref_out = torch.empty(M, N, device=dev)
    aux_r = torch.empty_like(aux)
    cs_r = torch.zeros(N, device=dev)
    _gemm_ref(a, b, True, True, ref_out, bias, 2, 1, z, aux_r, res, 1.0, None, False, cs_r)
    assert rel_err(out, ref_out) < 2e-3
    assert rel_err(aux, aux_r) < 1e-2
    assert rel_err(cs, cs_r) < 2e-3
    od_r = torch.empty(M, N, device=dev)
    cs2_r = torch.zeros(N, device=dev)
    _gemm_ref(a, b, True, True, od_r, None, 0, 2, z, None, None, 1.0, None, False, cs2_r)
    assert rel_err(od, od_r) < 1e-2
    assert rel_err(cs2, cs2_r) < 2e-3
    og_r = torch.empty(M, N, device=dev)
    _gemm_ref(a, b, True, True, og_r, bias, 2, 0, None, torch.empty_like(aux), None, 1.0, None, False)
    assert rel_err(og, og_r) < 1e-2


@pytest.mark.parametrize("M,N,K", [(1023, 768, 768), (16384, 3072, 192), (3000, 2312, 320)])
@pytest.mark.parametrize("with_bias", [True, False])
@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("out_f32", [False, True])
def test_gemm_v9_forward_epilogue(M, N, K, with_bias, act, out_f32):
    """v9's load-free forward epilogue (gemm9_kern.h EPI 1: bias staged into LDS by the operand
    DMA stream, activation, the pre-activation aux_out, 64 stores in flight into the next unit),
    forced by impl 26 on nt products: ragged M and N, 768 tiles at K = 192 (three units per
    persistent workgroup: the bias buffers of unit parity are reused), against f32 PyTorch."""
    torch.manual_seed(5)
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    A, B = _store(a, True), _store(b, True)
    bias = torch.randn(N, device=dev) if with_bias else None
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    _lib.set_gemm_impl(26)
    try:
        out = gemm(A, B, bias=bias, act=act, aux_out=aux, out_dtype=torch.float32 if out_f32 else torch.bfloat16)
        ran = _lib.gemm_last_kernel()
    finally:
        _lib.set_gemm_impl(-1)
    assert ran == 901, ran  # the v9 EPI 1 kernel itself, not a fallback
    ref = torch.empty(M, N, device=dev)
    aux_r = torch.empty_like(aux)
    _gemm_ref(a, b, True, True, ref, bias, act, 0, None, aux_r, None, 1.0, None, False)
    assert rel_err(out, ref) < (2e-3 if out_f32 else 1e-2)
    assert rel_err(aux, aux_r) < 1e-2
    assert _lib.is_loaded()


@pytest.mark.parametrize("act_bwd", [2, 3])
@pytest.mark.parametrize("act_lds", [0, 1])
@pytest.mark.parametrize("use_ws", [False, True])
@pytest.mark.parametrize("a_kmaj,b_kmaj", [(True, False), (True, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(1023, 768, 768), (4096, 4352, 256), (300, 264, 96), (2048, 3072, 512)])
def test_gemm_v7_act_grad_epilogue_paths(monkeypatch, act_bwd, act_lds, use_ws, a_kmaj, b_kmaj, M, N, K):
    """The v7 input-gradient epilogue (act' of a bf16 operand + bias-gradient column sums) on
    both paths: the act' operand staged through LDS in quarters (gemm7_kern.h
    g7_epilogue_act_lds, EPI 8; EPI 10 for ACT_MUL = 3, the operand already act'(z); column sums
    as per-tile partials in the workspace + a reduction, or f32 atomics without one) and the
    per-lane operand reads (DPC_G7_ACTLDS=0) -- ragged edge tiles, and more tiles than CUs
    (4096 x 4352: a workgroup streams two through its ring)."""
    from distributed_pytorch_cookbook_amd.ops import gemm as G

    if not use_ws:
        monkeypatch.setattr(G, "_workspace", lambda device: None)
    torch.manual_seed(5)
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    A, B = _store(a, a_kmaj), _store(b, b_kmaj)
    z = torch.randn(M, N, device=dev).bfloat16()
    lib = _lib.lib()
    _lib.set_gemm_impl(25)
    lib.dpc_gemm7_set_act_lds(act_lds)
    try:
        cs = torch.full((N,), 0.25, device=dev)
        od = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, act_bwd=act_bwd, aux_in=z, colsum=cs)
        ran = _lib.gemm_last_kernel()
        of = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, act_bwd=act_bwd, aux_in=z, out_dtype=torch.float32, alpha=0.5)
    finally:
        _lib.set_gemm_impl(-1)
        lib.dpc_gemm7_set_act_lds(-1)
    if act_lds and a_kmaj:  # the LDS-staged epilogue itself ran (EPI 8, or EPI 10 for ACT_MUL)
        assert ran == (710 if act_bwd == 3 else 708), ran
    od_r = torch.empty(M, N, device=dev)
    cs_r = torch.full((N,), 0.25, device=dev)
    _gemm_ref(a, b, True, True, od_r, None, 0, act_bwd, z, None, None, 1.0, None, False, cs_r)
    assert rel_err(od, od_r) < 1e-2
    assert rel_err(cs, cs_r) < 2e-3
    of_r = torch.empty(M, N, device=dev)
    _gemm_ref(a, b, True, True, of_r, None, 0, act_bwd, z, None, None, 0.5, None, False)
    assert rel_err(of, of_r) < 2e-3


@pytest.mark.parametrize("impl", [26, 25, 21, 10, 2])
@pytest.mark.parametrize("M,N,K", [(1023, 768, 768), (4096, 4352, 256), (300, 264, 192), (2048, 3072, 768)])
def test_gemm_aux_deriv_then_mul(impl, M, N, K):
    """The FFN pair of models/fused.py: the up-projection forward stores GELU'(z) as its second
    output (aux_deriv: v9 full-tile and edge copies, v7 / v8 generic MODE 1, v3 / v2 epi_tile) and
    the input gradient multiplies it in (ACT_MUL); against f32 PyTorch of the z-form chain
    (gelu'(z) evaluated from the f32 pre-activation)."""
    torch.manual_seed(7)
    a = torch.randn(M, K, device=dev).bfloat16() * 0.5
    b = torch.randn(N, K, device=dev).bfloat16() * 0.1
    bias = torch.randn(N, device=dev)
    A, B = _store(a, True), _store(b, True)
    g1 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dy = torch.randn(M, K, device=dev).bfloat16()
    Bn = _store(b, False)  # dz1 = (dy @ W) * g1: W stored [N, K] -> mn-major operand [K, N]
    _lib.set_gemm_impl(impl)
    try:
        u = gemm(A, B, bias=bias, act=2, aux_out=g1, aux_deriv=True)
        cs = torch.zeros(N, device=dev)
        dz = gemm(dy, Bn, a_kmaj=True, b_kmaj=False, act_bwd=3, aux_in=g1, colsum=cs)
    finally:
        _lib.set_gemm_impl(-1)
    z = a.float() @ b.float().t() + bias
    from distributed_pytorch_cookbook_amd.ops.gemm import act_grad_ref

    gd = act_grad_ref(z, 2)
    assert rel_err(g1, gd) < 1e-2
    assert rel_err(u, torch.nn.functional.gelu(z, approximate="tanh")) < 1e-2
    dz_r = (dy.float() @ b.float().t()) * gd
    assert rel_err(dz, dz_r) < 1.5e-2
    assert rel_err(cs, dz_r.sum(0)) < 1e-2


@pytest.mark.parametrize("res_lds", [0, 1])
@pytest.mark.parametrize("act,with_aux,with_bias", [(2, True, True), (0, False, True), (1, True, False)])
@pytest.mark.parametrize("a_kmaj,b_kmaj", [(True, True), (True, False)])
@pytest.mark.parametrize("M,N,K", [(1023, 768, 768), (4096, 4352, 256), (300, 264, 96)])
def test_gemm_v7_residual_epilogue_paths(res_lds, act, with_aux, with_bias, a_kmaj, b_kmaj, M, N, K):
    """The v7 forward epilogue into an f32 output with an f32 residual (the FFN down-projection:
    bias + GELU + pre-activation aux + residual) on both paths: the residual staged through LDS
    in 16-row eighths (gemm7_kern.h g7_epilogue_res_lds, EPI 9) and the per-lane reads
    (DPC_G7_RESLDS=0); the residual is also passed aliased to the output, as the model does."""
    torch.manual_seed(6)
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    A, B = _store(a, a_kmaj), _store(b, b_kmaj)
    bias = torch.randn(N, device=dev) if with_bias else None
    res = torch.randn(M, N, device=dev)
    lib = _lib.lib()
    _lib.set_gemm_impl(25)
    lib.dpc_gemm7_set_res_lds(res_lds)
    try:
        aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if with_aux else None
        out = gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, bias=bias, act=act, aux_out=aux, residual=res,
                   out_dtype=torch.float32, alpha=0.75)
        inplace = res.clone()
        gemm(A, B, a_kmaj=a_kmaj, b_kmaj=b_kmaj, bias=bias, act=act, residual=inplace, out=inplace, alpha=0.75)
    finally:
        _lib.set_gemm_impl(-1)
        lib.dpc_gemm7_set_res_lds(-1)
    ref = torch.empty(M, N, device=dev)
    aux_r = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if with_aux else None
    _gemm_ref(a, b, True, True, ref, bias, act, 0, None, aux_r, res, 0.75, None, False)
    assert rel_err(out, ref) < 2e-3
    assert rel_err(inplace, ref) < 2e-3
    if with_aux:
        assert rel_err(aux, aux_r) < 1e-2


@pytest.mark.parametrize("M,N,K", [(16000, 3072, 768), (12000, 2560, 1600), (10000, 2048, 576), (4096, 4352, 768),
                                   (65472, 3072, 768), (65472, 768, 3072), (9000, 1600, 2048)])
def test_gemm_v7d_deferred_gelu_epilogues(M, N, K):
    """impl 24 (gemm7.hip gemm7d_kernel): the FFN's GELU forward (bias + GELU + pre-activation,
    both operands k-major) and GELU' input gradient (act'(aux_in) + column sums, B n-major)
    with the element-wise half deferred into the next tile's main loop.  Shapes give every
    persistent workgroup 1-3+ tiles (deferred steady state, the last-tile and ragged-M
    fallbacks) at the three schedule regimes: nk = 18 (two chunks per slice), 24 (two, then
    one) and 50 (one, then none)."""
    torch.manual_seed(5)
    a = torch.randn(M, K, device=dev).bfloat16()
    b = torch.randn(N, K, device=dev).bfloat16()
    bias = torch.randn(N, device=dev)
    z = torch.randn(M, N, device=dev).bfloat16()
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=dev)
    A, Bk, Bn = _store(a, True), _store(b, True), _store(b, False)
    _lib.set_gemm_impl(24)
    try:
        og = gemm(A, Bk, a_kmaj=True, b_kmaj=True, bias=bias, act=2, aux_out=aux)
        od = gemm(A, Bn, a_kmaj=True, b_kmaj=False, act_bwd=2, aux_in=z, colsum=cs)
    finally:
        _lib.set_gemm_impl(-1)
    og_r = torch.empty(M, N, device=dev)
    aux_r = torch.empty_like(aux)
    _gemm_ref(a, b, True, True, og_r, bias, 2, 0, None, aux_r, None, 1.0, None, False)
    assert rel_err(aux, aux_r) < 1e-2
    assert rel_err(og, og_r) < 1e-2
    od_r = torch.empty(M, N, device=dev)
    cs_r = torch.zeros(N, device=dev)
    _gemm_ref(a, b, True, True, od_r, None, 0, 2, z, None, None, 1.0, None, False, cs_r)
    assert rel_err(od, od_r) < 1e-2
    assert rel_err(cs, cs_r) < 2e-3
    # every element written (no chunk skipped by the deferred schedule)
    assert torch.isfinite(og.float()).all() and torch.isfinite(od.float()).all()
    # the down projection (f32 residual in, f32 out; deferred at K >= 1088)
    res = torch.randn(M, N, device=dev)
    aux2 = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    _lib.set_gemm_impl(24)
    try:
        ox = gemm(A, Bk, a_kmaj=True, b_kmaj=True, bias=bias, act=2, aux_out=aux2, residual=res,
                  out_dtype=torch.float32)
    finally:
        _lib.set_gemm_impl(-1)
    ox_r = torch.empty(M, N, device=dev)
    aux2_r = torch.empty_like(aux2)
    _gemm_ref(a, b, True, True, ox_r, bias, 2, 0, None, aux2_r, res, 1.0, None, False)
    assert rel_err(aux2, aux2_r) < 1e-2
    assert rel_err(ox, ox_r) < 5e-3


@pytest.mark.parametrize("impl", [2, 4, 10, 16, 21, 25, 26])
@pytest.mark.parametrize("splits", [2, 3, 8])
@pytest.mark.parametrize("M,N,K", [(77, 1000, 4160), (600, 520, 8192), (2304, 136, 4096)])
def test_gemm_forced_split_k(impl, splits, M, N, K):
    """Split-K partial sums (lane-contiguous atomic epilogue) on ragged M/N edges."""
    torch.manual_seed(5)
    A = torch.randn(K, (M + 7) // 8 * 8, device=dev).bfloat16()[:, :M]
    B = torch.randn(K, (N + 7) // 8 * 8, device=dev).bfloat16()[:, :N]
    acc0 = torch.randn(M, N, device=dev)
    acc = acc0.clone()
    _lib.set_gemm_impl(impl)
    _lib.set_gemm_splits(splits)
    try:
        gemm(A, B, a_kmaj=False, b_kmaj=False, out=acc, accumulate=True)
        fresh = gemm(A, B, a_kmaj=False, b_kmaj=False, out_dtype=torch.float32)
    finally:
        _lib.set_gemm_impl(-1)
        _lib.set_gemm_splits(0)
    ref = A.float().t() @ B.float()
    assert rel_err(acc - acc0, ref) < 2e-3
    assert rel_err(fresh, ref) < 2e-3


def test_gemm_identity_asymmetric():
    # A = I with an asymmetric B catches a transposed C write
    n = 128
    a = torch.eye(n, device=dev).bfloat16()
    b = torch.arange(n * n, device=dev).reshape(n, n).float().remainder(251).bfloat16()
    out = gemm(a, b, out_dtype=torch.float32)
    assert torch.equal(out, b.float().t())


@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm_epilogues(act):
    torch.manual_seed(1)
    M, N, K = 333, 264, 192
    a = torch.randn(M, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16() * 0.1
    bias = torch.randn(N, device=dev)
    res = torch.randn(M, N, device=dev)
    aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    out = gemm(a, w, bias=bias, act=act, residual=res, aux_out=aux, out_dtype=torch.float32)
    aux_r = torch.empty_like(aux)
    ref = _gemm_ref(a, w, True, True, torch.empty(M, N, device=dev), bias, act, 0, None, aux_r, res,
                    1.0, None, False)
    assert rel_err(out, ref) < 2e-3
    assert rel_err(aux, aux_r) < 1e-2
    # act-backward epilogue + accumulate into f32
    z = torch.randn(M, N, device=dev).bfloat16()
    acc0 = torch.randn(M, N, device=dev)
    acc = acc0.clone()
    gemm(a, w, act_bwd=act, aux_in=z, out=acc, accumulate=True)
    ref2 = acc0.clone()
    _gemm_ref(a, w, True, True, ref2, None, 0, act, z, None, None, 1.0, None, True)
    assert rel_err(acc, ref2) < 2e-3


@pytest.mark.parametrize("hd", [64, 32, 128])
@pytest.mark.parametrize("S", [1023, 200, 64])
@pytest.mark.parametrize("with_pad", [False, True])
def test_attention_fwd_bwd(S, with_pad, hd, monkeypatch):
    """Native head sizes 32 / 64 / 128 (no pad path) against the f32 O(S^2) reference."""
    import distributed_pytorch_cookbook_amd.ops.attention as attn_mod

    def _no_pad(*a, **k):
        raise AssertionError("native head_dim must not take the zero-pad path")

    monkeypatch.setattr(attn_mod, "_pad_heads", _no_pad)
    torch.manual_seed(2)
    N, H = 2, 3
    T = N * S
    qkv = (torch.randn(T, 3 * H * hd, device=dev)).bfloat16()
    pad = None
    if with_pad:
        pad = torch.zeros(N, S, dtype=torch.bool, device=dev)
        pad[0, S - S // 4:] = True  # right padding
        pad[1, 5:9] = True
    o, lse = attention_fwd(qkv, N, S, H, hd, pad, causal=True)
    o_r, lse_r = attention_ref(qkv, N, S, H, hd, pad, causal=True)
    assert rel_err(o, o_r) < 1e-2
    fin = torch.isfinite(lse_r)
    assert torch.allclose(lse[fin], lse_r[fin], atol=2e-2, rtol=1e-3)
    do = torch.randn(T, H * hd, device=dev).bfloat16()
    dqkv = attention_bwd(do, qkv, o, lse, N, S, H, hd, pad, causal=True)
    x = qkv.float().requires_grad_(True)
    o_ref, _ = attention_ref(x, N, S, H, hd, pad, causal=True)
    (g,) = torch.autograd.grad(o_ref, x, do.float())
    for i, name in enumerate("qkv"):
        sl = slice(i * H * hd, (i + 1) * H * hd)
        assert rel_err(dqkv[:, sl], g[:, sl]) < 2e-2, name


@pytest.mark.parametrize("hd", [64, 32])
@pytest.mark.parametrize("S", [4096, 8191])
def test_attention_long_context(S, hd):
    """O(S) flash attention at 4-8x GPT-2's context, vs the f32 O(S^2) reference."""
    torch.manual_seed(5)
    N, H = 1, 2
    qkv = torch.randn(N * S, 3 * H * hd, device=dev).bfloat16()
    o, lse = attention_fwd(qkv, N, S, H, hd, None, causal=True)
    o_r, lse_r = attention_ref(qkv, N, S, H, hd, None, causal=True)
    assert rel_err(o, o_r) < 1e-2
    assert torch.allclose(lse, lse_r, atol=2e-2, rtol=1e-3)
    do = torch.randn_like(o)
    dqkv = attention_bwd(do, qkv, o, lse, N, S, H, hd, None, causal=True)
    x = qkv.float().requires_grad_(True)
    (g,) = torch.autograd.grad(attention_ref(x, N, S, H, hd, None, causal=True)[0], x, do.float())
    for i, name in enumerate("qkv"):
        sl = slice(i * H * hd, (i + 1) * H * hd)
        assert rel_err(dqkv[:, sl], g[:, sl]) < 2e-2, name


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("hd", [16, 48, 32, 96, 160])
def test_attention_head_dim_other(hd, causal):
    """Head sizes without a kernel of their own run zero-padded to the next one (16 -> 32,
    48 -> 64, 96 -> 128); past the largest kernel (160) the device runs the reference math
    (/root/reference/models/gpt.py:44-66 takes any head_dim); also the non-causal form."""
    torch.manual_seed(3)
    N, S, H = 2, 100, 4
    qkv = torch.randn(N * S, 3 * H * hd, device=dev).bfloat16()
    o, lse = attention_fwd(qkv, N, S, H, hd, causal=causal)
    o_r, _ = attention_ref(qkv, N, S, H, hd, causal=causal)
    assert rel_err(o, o_r) < 1e-2
    do = torch.randn_like(o)
    d = attention_bwd(do, qkv, o, lse, N, S, H, hd, causal=causal)
    x = qkv.float().requires_grad_(True)
    (g,) = torch.autograd.grad(attention_ref(x, N, S, H, hd, causal=causal)[0], x, do.float())
    assert rel_err(d, g) < 2e-2


def test_attention_bwd_block_order_bitwise():
    """The backward's block order (DPC_ATTN_ORDER: 1 heaviest-first over the grid, 0 per-XCD
    head-major) only changes WHEN each workgroup runs, not what it sums: dQ / dK / dV are bitwise
    equal under both."""
    from distributed_pytorch_cookbook_amd.ops import _lib
    torch.manual_seed(21)
    N, S, H, hd = 2, 300, 3, 64
    qkv = (torch.randn(N * S, 3 * H * hd, device=dev) * 0.5).bfloat16()
    o, lse = attention_fwd(qkv, N, S, H, hd, causal=True)
    do = torch.randn_like(o)
    outs = []
    try:
        for order in (1, 0):
            _lib.lib().dpc_attn_set_order(order)
            outs.append(attention_bwd(do, qkv, o, lse, N, S, H, hd, causal=True).clone())
    finally:
        _lib.lib().dpc_attn_set_order(-1)
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("pf", [1, 0])
@pytest.mark.parametrize("D", [100, 256, 768, 1600])
def test_layernorm(D, pf):
    """pf: the backward's next-row prefetch on / off (DPC_LN_BWD_PF); D = 100 and 1600 leave lanes
    past the row end (the clamped, unconditional loads)."""
    from distributed_pytorch_cookbook_amd.ops import _lib
    _lib.lib().dpc_layernorm_set_bwd_prefetch(pf)
    try:
        _test_layernorm(D)
    finally:
        _lib.lib().dpc_layernorm_set_bwd_prefetch(-1)


def _test_layernorm(D):
    torch.manual_seed(4)
    T = 517
    x = torch.randn(T, D, device=dev) * 3 + 1
    g = torch.randn(D, device=dev)
    b = torch.randn(D, device=dev)
    y, mean, rstd = layernorm_fwd(x, g, b)
    yr = torch.nn.functional.layer_norm(x, (D,), g, b, 1e-5)
    assert rel_err(y, yr) < 5e-3
    dy = torch.randn(T, D, device=dev)
    dres = torch.randn(T, D, device=dev)
    dx = dres.clone()
    dg = torch.zeros(D, device=dev)
    db = torch.zeros(D, device=dev)
    layernorm_bwd(dy, x, mean, rstd, g, dx, dg, db)
    dx_only = torch.full_like(dx, float("nan"))  # dx_set: the old contents are never read
    layernorm_bwd(dy, x, mean, rstd, g, dx_only, torch.zeros(D, device=dev), torch.zeros(D, device=dev), dx_set=True)
    xx = x.clone().requires_grad_(True)
    gg = g.clone().requires_grad_(True)
    bb = b.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xx, (D,), gg, bb, 1e-5).backward(dy)
    assert rel_err(dx - dres, xx.grad) < 1e-4
    assert rel_err(dx_only, xx.grad) < 1e-4
    assert rel_err(dg, gg.grad) < 1e-4
    assert rel_err(db, bb.grad) < 1e-4
    # fused consumer: gout = bf16(dx * keep), gsum += colsum(dx * keep)
    from distributed_pytorch_cookbook_amd.ops.dropout import DropSpec, keep_mask
    for drop in (None, DropSpec.make(0.2, seed=3, site=5)):
        dx2 = dres.clone()
        gout = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
        gsum = torch.ones(D, device=dev)
        layernorm_bwd(dy, x, mean, rstd, g, dx2, torch.zeros(D, device=dev), torch.zeros(D, device=dev),
                      gout=gout, gsum=gsum, drop=drop)
        ref = dx2 if drop is None else dx2 * keep_mask(drop, T, D, dev)
        assert rel_err(gout, ref) < 5e-3
        assert rel_err(gsum - 1, ref.sum(0)) < 1e-4
    # ... with an activation in front of the dropout (the previous layer's FFN tail):
    # gout = bf16(dx * keep * act'(z))
    from distributed_pytorch_cookbook_amd.ops.gemm import act_grad_ref
    z = (torch.randn(T, D, device=dev) * 2).bfloat16()
    for act in (1, 2):
        for drop in (None, DropSpec.make(0.2, seed=7, site=1)):
            dx2 = dres.clone()
            gout = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
            gsum = torch.zeros(D, device=dev)
            layernorm_bwd(dy, x, mean, rstd, g, dx2, torch.zeros(D, device=dev), torch.zeros(D, device=dev),
                          gout=gout, gsum=gsum, drop=drop, gz=z, gact=act)
            ref = dx2 * act_grad_ref(z.float(), act)
            if drop is not None:
                ref = ref * keep_mask(drop, T, D, dev)
            assert rel_err(gout, ref) < 5e-3, act
            assert rel_err(gsum, ref.sum(0)) < 1e-4, act
    # bf16 dy (the input gradient of the next Linear): same math on the rounded values
    dyb = dy.bfloat16()
    dx3 = dres.clone()
    dg3, db3 = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    layernorm_bwd(dyb, x, mean, rstd, g, dx3, dg3, db3)
    xx.grad, gg.grad, bb.grad = None, None, None
    torch.nn.functional.layer_norm(xx, (D,), gg, bb, 1e-5).backward(dyb.float())
    assert rel_err(dx3 - dres, xx.grad) < 1e-4
    assert rel_err(dg3, gg.grad) < 1e-4
    assert rel_err(db3, bb.grad) < 1e-4


@pytest.mark.parametrize("tdt", [torch.float32, torch.bfloat16])
def test_embedding(tdt):
    torch.manual_seed(5)
    V, P, D, T = 1000, 64, 768, 4 * 63
    tok = torch.randn(V, D, device=dev).to(tdt)
    pt = torch.randn(P, D, device=dev).to(tdt)
    ids = torch.randint(0, V, (T,), device=dev)
    pos = torch.arange(63, device=dev).repeat(4)
    x = embedding_fwd(ids, pos, tok, pt)
    assert torch.allclose(x, tok[ids].float() + pt[pos].float(), atol=1e-6)
    dx = torch.randn(T, D, device=dev)
    dt = torch.zeros(V, D, device=dev)
    dp = torch.zeros(P, D, device=dev)
    embedding_bwd(dx, ids, pos, dt, dp)
    rt = torch.zeros(V, D, device=dev).index_add_(0, ids, dx)
    rp = torch.zeros(P, D, device=dev).index_add_(0, pos, dx)
    assert torch.allclose(dt, rt, atol=1e-4) and torch.allclose(dp, rp, atol=1e-4)


@pytest.mark.parametrize("D", [64, 768, 1600])
def test_embedding_bwd_deterministic(D):
    """The sorted embedding backward (csrc/embed_bwd.hip): equals an f64 index_add, accumulates
    into existing gradients, skips out-of-range ids, and is bitwise identical across runs even
    with heavily repeated ids (the atomic scatter is not)."""
    from distributed_pytorch_cookbook_amd.ops import embedding as emb
    torch.manual_seed(9)
    V, P, S, N = 5000, 1024, 1023, 8
    T = N * S
    ids = torch.randint(0, 40, (T,), device=dev)  # ~200 repeats per id
    ids[::97] = torch.randint(0, V, (ids[::97].numel(),), device=dev)
    ids[5] = V + 3  # out of range: ignored
    pos = torch.arange(S, device=dev).repeat(N)
    dx = torch.randn(T, D, device=dev)
    base_t, base_p = torch.randn(V, D, device=dev), torch.randn(P, D, device=dev)
    outs = []
    for _ in range(2):
        dt, dp = base_t.clone(), base_p.clone()
        emb.embedding_bwd(dx, ids, pos, dt, dp)
        outs.append((dt, dp))
    assert emb._ws, "the sorted path did not run"
    ok = ids < V
    rt = base_t.double().index_add_(0, ids[ok], dx[ok].double())
    rp = base_p.double().index_add_(0, pos, dx.double())
    assert torch.allclose(outs[0][0].double(), rt, atol=2e-4, rtol=1e-5)
    assert torch.allclose(outs[0][1].double(), rp, atol=2e-4, rtol=1e-5)
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("V,mode", [(50257, 0), (1000, 0), (9000, 0), (40000, 0), (70001, 0),
                                    (50257, 1), (50257, 2)])
def test_cross_entropy(V, mode):
    """Register-resident rows (ce_kernel<1..16>: V = 1000 .. 50257), the streaming fallback
    (V = 70001 > 64K columns) and the forced streaming modes, all in place."""
    torch.manual_seed(6)
    T = 300
    ld = (V + 63) // 64 * 64
    _lib.lib().dpc_ce_set_mode(mode)
    buf = torch.zeros(T, ld, device=dev, dtype=torch.bfloat16)
    buf[:, :V] = (torch.randn(T, V, device=dev) * 2).bfloat16()
    logits = buf.clone()
    tg = torch.randint(0, V, (T,), device=dev)
    tg[::7] = -100
    try:
        loss, n, correct = cross_entropy_fused(buf, tg, V, write_grad=True, want_correct=True)
    finally:
        _lib.lib().dpc_ce_set_mode(-1)
    lf = logits[:, :V].float().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(lf, tg, ignore_index=-100)
    lr.backward()
    assert abs(loss.item() - lr.item()) < 1e-3 * abs(lr.item())
    assert rel_err(buf[:, :V], lf.grad) < 1e-2
    assert ld == V or buf[:, V:].abs().max().item() == 0
    valid = tg != -100
    rc = (lf.argmax(-1) == tg)[valid].sum().item()
    assert abs(correct.item() - rc) <= 1


@pytest.mark.parametrize("V", [50257, 1000])
def test_cross_entropy_minus_inf_chunks(V):
    """Rows holding whole 8-aligned chunks of -inf logits (e.g. a masked vocabulary range): the
    chunk adds nothing to the row's sum-exp (no NaN from -inf - -inf), as in torch."""
    torch.manual_seed(8)
    T = 64
    ld = (V + 63) // 64 * 64
    buf = torch.zeros(T, ld, device=dev, dtype=torch.bfloat16)
    buf[:, :V] = torch.randn(T, V, device=dev).bfloat16()
    buf[::2, 16:40] = float("-inf")           # three whole chunks (16..39) on even rows
    buf[1::4, 8 * 37:8 * 40] = float("-inf")  # and three more on every fourth row
    logits = buf.clone()
    tg = torch.randint(40, V, (T,), device=dev)
    loss, n, correct = cross_entropy_fused(buf, tg, V, write_grad=True, want_correct=True)
    lf = logits[:, :V].float().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(lf, tg)
    lr.backward()
    assert torch.isfinite(loss).item()
    assert abs(loss.item() - lr.item()) < 1e-3 * abs(lr.item())
    assert torch.isfinite(buf[:, :V].float()).all()
    assert rel_err(buf[:, :V], lf.grad) < 1e-2


def test_gemm_autotune_leaves_outputs_intact():
    """The autotuner times candidates on CLONES of the outputs: an accumulating weight
    gradient and a column-sum epilogue must come out exactly as one untuned call makes them."""
    from distributed_pytorch_cookbook_amd.ops import gemm as G
    torch.manual_seed(12)
    T, N, K = 4096, 384, 256
    dy = torch.randn(T, N, device=dev).bfloat16()
    x = torch.randn(T, K, device=dev).bfloat16()
    g0 = torch.randn(N, K, device=dev)
    z = torch.randn(T, K, device=dev).bfloat16()
    w = torch.randn(N, K, device=dev).bfloat16()
    saved = (G._TUNE, dict(G._table), dict(G._tuned_new))
    try:
        G._TUNE, G._table, G._tuned_new = True, {}, {}
        g = g0.clone()
        G.gemm(dy, x, a_kmaj=False, b_kmaj=False, out=g, accumulate=True)
        cs = torch.zeros(K, device=dev)
        d = G.gemm(dy, w, a_kmaj=True, b_kmaj=False, act_bwd=2, aux_in=z, colsum=cs)
        assert len(G._tuned_new) == 2 and all(v in G._CANDIDATES for v in G._tuned_new.values())
    finally:
        G._TUNE, G._table, G._tuned_new = saved
    assert rel_err(g - g0, dy.float().t() @ x.float()) < 2e-3
    d_r = torch.empty(T, K, device=dev)
    cs_r = torch.zeros(K, device=dev)
    _gemm_ref(dy, w.t().contiguous(), True, True, d_r, None, 0, 2, z, None, None, 1.0, None, False, cs_r)
    assert rel_err(d, d_r) < 1e-2 and rel_err(cs, cs_r) < 2e-3


def test_adamw_matches_torch():
    torch.manual_seed(7)
    n = 4096
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
    opt = FlatAdamW(p, g, lr=1e-3, shadow=sh)
    pr = p.clone().requires_grad_(True)
    ref = torch.optim.AdamW([pr], lr=1e-3)
    for _ in range(3):
        g.normal_()
        pr.grad = g.clone()
        opt.step()
        ref.step()
    assert rel_err(p, pr.detach()) < 1e-6
    assert rel_err(sh, pr.detach()) < 5e-3


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("N", [3072, 772])
def test_bias_act_bwd(act, N):
    torch.manual_seed(8)
    T = 777
    dy = torch.randn(T, N, device=dev)
    z = torch.randn(T, N, device=dev).bfloat16()
    db = torch.zeros(N, device=dev)
    dz = bias_act_bwd(dy, z, act, db)
    db_r = torch.zeros(N, device=dev)
    dz_r = bias_act_bwd(dy.cpu(), z.cpu(), act, db_r.cpu().clone(), out_dtype=torch.float32)
    from distributed_pytorch_cookbook_amd.ops.gemm import act_grad_ref
    ref = dy * act_grad_ref(z, act) if act else dy
    assert rel_err(dz, ref) < 5e-3
    assert rel_err(db, ref.sum(0)) < 1e-4
    assert dz_r.shape == dz.shape


def test_native_library_loaded():
    assert _lib.is_loaded()


@pytest.mark.parametrize("impl", [1, 2, 10])
def test_gemm_padded_vocab_head(impl):
    """lm_head over a 64-padded vocab: B has V < N rows (read as zeros), and the dgrad runs
    with K = padded vocab while W_lm holds only V k-rows."""
    torch.manual_seed(12)
    T, D, V = 300, 256, 1001
    ld = (V + 63) // 64 * 64
    h = torch.randn(T, D, device=dev).bfloat16()
    w = torch.randn(V, D, device=dev).bfloat16()
    _lib.set_gemm_impl(impl)
    try:
        buf = torch.full((T, ld), 7.0, device=dev).bfloat16()
        gemm(h, w, out=buf)
        g = torch.zeros(T, ld, device=dev).bfloat16()
        g[:, :V] = torch.randn(T, V, device=dev).bfloat16()
        dh = gemm(g, w, a_kmaj=True, b_kmaj=False, out_dtype=torch.float32)
        # split-K plain f32 product (wgrad shape) with and without accumulate
        dy = torch.randn(8192, 256, device=dev).bfloat16()
        x = torch.randn(8192, 128, device=dev).bfloat16()
        o1 = gemm(dy, x, a_kmaj=False, b_kmaj=False, out_dtype=torch.float32)
        o2 = torch.ones(256, 128, device=dev)
        gemm(dy, x, a_kmaj=False, b_kmaj=False, out=o2, accumulate=True)
    finally:
        _lib.set_gemm_impl(-1)
    ref = h.float() @ w.float().t()
    assert rel_err(buf[:, :V], ref) < 1e-2
    assert buf[:, V:].abs().max().item() == 0
    assert rel_err(dh, g[:, :V].float() @ w.float()) < 2e-3
    r = dy.float().t() @ x.float()
    assert rel_err(o1, r) < 2e-3 and rel_err(o2 - 1, r) < 2e-3


def test_dropout_kernels_match_torch_twin():
    """The device hash mask is bit-identical to ops/dropout.py:keep_mask."""
    from distributed_pytorch_cookbook_amd.ops.dropout import DropSpec, dropout_residual, keep_mask

    torch.manual_seed(13)
    T, N = 1031, 768
    spec = DropSpec.make(0.1, seed=(5 << 32) | 17, site=9)
    y = torch.randn(T, N, device=dev)
    r = torch.randn(T, N, device=dev)
    out = dropout_residual(y, r, spec)
    keep = keep_mask(spec, T, N, dev)
    assert torch.equal(out == r, (keep == 0) | (y == 0))
    assert rel_err(out, r + y * keep) < 1e-6
    # in place, aliasing y
    y2 = y.clone()
    dropout_residual(y2, r, spec, out=y2)
    assert torch.equal(y2, out)
    # backward: dz = dy * keep * act'(z)
    from distributed_pytorch_cookbook_amd.ops.gemm import act_grad_ref
    z = torch.randn(T, N, device=dev).bfloat16()
    db = torch.zeros(N, device=dev)
    dz = bias_act_bwd(y, z, 2, db, drop=spec)
    ref = y * keep * act_grad_ref(z, 2)
    assert rel_err(dz, ref) < 5e-3
    assert rel_err(db, ref.sum(0)) < 1e-4
    assert torch.equal(dz == 0, (ref == 0))


@pytest.mark.parametrize("D,p_drop", [(768, 0.0), (1600, 0.0), (768, 0.1)])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_layernorm_fwd_fused_residual_add(D, p_drop, act):
    """LN forward with the projection's bias + activation + dropout + residual add fused in:
    xs = x + keep * act(y + b) written to x_out, LN(xs) vs the torch expression (act: the FFN
    down projection's ReLU / GELU, whose residual add the next layer's LN1 now does)."""
    from distributed_pytorch_cookbook_amd.ops.dropout import DropSpec, keep_mask
    from distributed_pytorch_cookbook_amd.ops.gemm import act_fwd_ref
    torch.manual_seed(13)
    T = 1000
    x = torch.randn(T, D, device=dev)
    y = torch.randn(T, D, device=dev).bfloat16()
    b = torch.randn(D, device=dev)
    g, be = torch.randn(D, device=dev), torch.randn(D, device=dev)
    drop = DropSpec.make(p_drop, seed=5, site=3) if p_drop else None
    xs = torch.empty(T, D, device=dev)
    h, mu, rs = layernorm_fwd(x, g, be, 1e-5, torch.bfloat16, add=(y, b, drop, act), x_out=xs)
    a = act_fwd_ref(y.float() + b, act)
    if drop is not None:
        a = a * keep_mask(drop, T, D, dev)
    xs_r = x + a
    assert rel_err(xs, xs_r) < (1e-6 if act != 2 else 1e-5)
    h_r = torch.nn.functional.layer_norm(xs_r, (D,), g, be, 1e-5)
    assert rel_err(h, h_r) < 1e-2
    assert rel_err(mu, xs_r.mean(-1)) < 1e-5


@pytest.mark.parametrize("hd", [64, 32, 128, 96, 256])
@pytest.mark.parametrize("pos", [0, 37, 299])
def test_decode_attention(hd, pos):
    """Single-query KV-cache attention kernel (appends the new K/V at the device length) vs
    the f32 softmax over the cached keys."""
    from distributed_pytorch_cookbook_amd.ops.attention import decode_attention

    torch.manual_seed(7)
    N, H, Smax = 2, 3, 300
    E = H * hd
    kc = torch.randn(N, Smax, E, device=dev).bfloat16()
    vc = torch.randn(N, Smax, E, device=dev).bfloat16()
    kc[:, pos:] = 0  # not yet written
    vc[:, pos:] = 0
    qkv = torch.randn(N, 3 * E, device=dev).bfloat16()
    length = torch.full((1,), pos, device=dev, dtype=torch.int64)
    k_ref, v_ref = kc.clone(), vc.clone()
    o = decode_attention(qkv, kc, vc, length, H, hd)
    k_ref[:, pos] = qkv[:, E:2 * E]
    v_ref[:, pos] = qkv[:, 2 * E:]
    assert torch.equal(kc, k_ref) and torch.equal(vc, v_ref)
    L = pos + 1
    q = qkv[:, :E].float().reshape(N, H, 1, hd)
    k = k_ref[:, :L].float().reshape(N, L, H, hd).transpose(1, 2)
    v = v_ref[:, :L].float().reshape(N, L, H, hd).transpose(1, 2)
    ref = (torch.softmax(q @ k.transpose(-1, -2) / math.sqrt(hd), -1) @ v).reshape(N, E)
    assert rel_err(o, ref) < 1e-2


@pytest.mark.parametrize("M", [1, 3, 8, 16])
@pytest.mark.parametrize("Nw,N,K", [(2304, 2304, 768), (50257, 50304, 768), (1600, 1600, 6400), (100, 104, 64)])
@pytest.mark.parametrize("epi", ["plain", "bias_gelu", "bias_relu_res"])
def test_gemv_few_rows(M, Nw, N, K, epi):
    """Decode-shaped Linear (csrc/decode.hip: dpc_gemv) against an f32 torch product of the same
    bf16 operands: bias / activation / f32 residual epilogue fused, padded output columns
    (N > weight rows) written as 0."""
    from distributed_pytorch_cookbook_amd.ops.gemm import _linear_fwd_few_rows, act_fwd_ref
    torch.manual_seed(7)
    x = torch.randn(M, K, device=dev).bfloat16()
    w = (torch.randn(Nw, K, device=dev) / K ** 0.5).bfloat16()
    bias = torch.randn(Nw, device=dev) if epi != "plain" else None
    act = {"plain": 0, "bias_gelu": 2, "bias_relu_res": 1}[epi]
    res = torch.randn(M, N, device=dev) if epi == "bias_relu_res" else None
    odt = torch.float32 if res is not None else torch.bfloat16
    out = torch.full((M, N), 7.0, device=dev, dtype=odt)
    y = _linear_fwd_few_rows(x, w, bias, act, res, out, odt)
    ref = x.float() @ w.float().t()
    if bias is not None:
        ref = ref + bias
    ref = act_fwd_ref(ref, act)
    if res is not None:
        ref = ref + res[:, :Nw]
    assert y is out
    assert rel_err(y[:, :Nw], ref) < (2e-3 if odt == torch.float32 else 1e-2)
    if N > Nw:
        assert torch.count_nonzero(y[:, Nw:]) == 0
