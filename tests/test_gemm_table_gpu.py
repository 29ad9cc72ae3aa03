"""Every product signature the training recipes dispatch (ops/gemm_tuned.json) against an fp32
reference of the same bf16 operands -- at its production size, with the implementation the
table picks for it (split-K counts, 256x256 persistent tiles, fused epilogues included).

The signature ``MxNxK:<a><b>:<out>:<act><act_bwd>:<flags>`` fixes the layouts (k = k-major,
m = mn-major), the output dtype (f = f32, h = bf16), the activation codes and the fused
operations (b = bias, x = pre-activation aux_out, r = f32 residual, c = bias-gradient column
sums, a = accumulate into C).  The error is measured per output against an fp32 product of
the bf16-rounded operands (the relative max error over the tile of the largest magnitude).
Reference: /root/reference/models/gpt.py:10-41 (the layers these products implement).
"""
import json
import os
import zlib

import pytest
import torch

from distributed_pytorch_cookbook_amd.ops import gemm as gemm_mod
from distributed_pytorch_cookbook_amd.ops.gemm import _gemm_ref, gemm

pytestmark = pytest.mark.gpu
dev = "cuda"

_TABLE = os.path.join(os.path.dirname(gemm_mod.__file__), "gemm_tuned.json")
with open(_TABLE) as f:
    SIGS = sorted(json.load(f)["impl"])


def _parse(sig):
    dims, lay, out, acts, flags = sig.split(":")
    M, N, K = (int(x) for x in dims.split("x"))
    return M, N, K, lay[0] == "k", lay[1] == "k", out == "f", int(acts[0]), int(acts[1]), flags


def _rel(x, ref):
    return float((x.float() - ref.float()).abs().max() / ref.float().abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("sig", SIGS)
def test_table_signature_matches_fp32(sig):
    M, N, K, a_kmaj, b_kmaj, out_f32, act, act_bwd, flags = _parse(sig)
    g = torch.Generator(device=dev).manual_seed(zlib.crc32(sig.encode()))

    def r(rows, cols):
        # production operands keep 16-B aligned rows (e.g. the 64-padded vocabulary of the LM
        # head): pad the row stride to a multiple of 64 elements and view the logical extent
        ld = (cols + 63) // 64 * 64
        return (torch.rand(rows, ld, device=dev, generator=g) * 2 - 1).bfloat16()[:, :cols]

    a = r(M, K) if a_kmaj else r(K, M)
    b = r(N, K) if b_kmaj else r(K, N)
    odt = torch.float32 if out_f32 else torch.bfloat16
    kw = {}
    if "b" in flags:
        kw["bias"] = torch.randn(N, device=dev, generator=g)
    if act:
        kw["act"] = act
    if "x" in flags:
        kw["aux_out"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if "r" in flags:
        kw["residual"] = torch.randn(M, N, device=dev, generator=g)
    if act_bwd:
        kw["act_bwd"] = act_bwd
        kw["aux_in"] = torch.randn(M, N, device=dev, generator=g).bfloat16()
    if "c" in flags:
        kw["colsum"] = torch.zeros(N, device=dev)
    accumulate = "a" in flags
    out = (torch.randn(M, N, device=dev, generator=g) if accumulate else torch.empty(M, N, device=dev)).to(odt)
    out0 = out.clone() if accumulate else None
    # the table lookup inside gemm() picks this signature's implementation
    assert gemm_mod._sig(M, N, K, a_kmaj, b_kmaj, out_f32, kw.get("bias"), act, act_bwd, kw.get("aux_out"),
                         kw.get("residual"), kw.get("colsum"), accumulate) == sig
    gemm(a, b, a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=out, accumulate=accumulate, **kw)
    torch.cuda.synchronize()

    ref = (out0.float() if accumulate else torch.empty(M, N, device=dev))
    ref_aux = torch.empty(M, N, device=dev) if "x" in flags else None
    ref_cs = torch.zeros(N, device=dev) if "c" in flags else None
    _gemm_ref(a, b, a_kmaj, b_kmaj, ref, kw.get("bias"), act, act_bwd, kw.get("aux_in"), ref_aux,
              kw.get("residual"), 1.0, None, accumulate, ref_cs)
    # bf16 outputs carry 2^-9 relative rounding; the f32 accumulation order differs over K
    tol = 1.5e-2 if not out_f32 else 5e-3
    assert _rel(out, ref) < tol, sig
    if ref_aux is not None:
        assert _rel(kw["aux_out"], ref_aux) < 1.5e-2, sig + " aux_out"
    if ref_cs is not None:
        assert _rel(kw["colsum"], ref_cs) < 5e-3, sig + " colsum"


@pytest.mark.parametrize("reserve", [16, 200])
@pytest.mark.parametrize("case", ["nt_v7", "nt_v8", "nn_v7", "tn_split", "fused_v7"])
def test_cu_reserve_products_match_fp32(reserve, case):
    """The persistent GEMMs with a resident-CU reserve (grid = CUs - reserve, the tiles spread
    over fewer workgroups, the split-K count re-planned) still match an fp32 product."""
    from distributed_pytorch_cookbook_amd.ops import _lib

    g = torch.Generator(device=dev).manual_seed(reserve + len(case))
    r = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).bfloat16()  # noqa: E731
    M, N, K = 4096, 2304, 768
    kw = {}
    if case == "tn_split":
        M, N, K = 2304, 768, 16384
        a, b = r(K, M), r(K, N)
        kw = dict(a_kmaj=False, b_kmaj=False, out_dtype=torch.float32)
        ref = a.float().t() @ b.float()
    elif case == "nn_v7":
        a, b = r(M, K), r(K, N)
        kw = dict(b_kmaj=False)
        ref = a.float() @ b.float()
    else:
        a, b = r(M, K), r(N, K)
        ref = a.float() @ b.float().t()
    impl = {"nt_v7": 20, "nt_v8": 21, "nn_v7": 20, "tn_split": -1, "fused_v7": 20}[case]
    if case == "fused_v7":
        bias = torch.randn(N, device=dev, generator=g)
        kw = dict(bias=bias, act=2)
        ref = torch.nn.functional.gelu(ref + bias, approximate="tanh")
    try:
        _lib.set_cu_reserve(reserve)
        _lib.set_gemm_impl(impl)
        out = gemm(a, b, **kw)
        torch.cuda.synchronize()
    finally:
        _lib.set_gemm_impl(-1)
        _lib.set_cu_reserve(0)
    assert _lib.get_cu_reserve() == 0
    assert _rel(out, ref) < 1e-2, _rel(out, ref)


@pytest.mark.parametrize("impl", [22, 23])
@pytest.mark.parametrize("lay", ["nt", "nn", "tn", "tt"])
def test_paired_dma_variant_matches_fp32(lay, impl):
    """v7 with the paired LDS-DMA issue (impl 22: one M0 write per two pieces, the second
    placed by the instruction offset) on every operand layout, edge tiles included."""
    from distributed_pytorch_cookbook_amd.ops import _lib

    g = torch.Generator(device=dev).manual_seed(22)
    r = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).bfloat16()  # noqa: E731
    M, N, K = 1000, 776, 1536
    a = r(M, K) if lay[0] == "n" else r(K, M)
    b = r(N, K) if lay[1] == "t" else r(K, N)
    am = a.float() if lay[0] == "n" else a.float().t()
    bm = b.float().t() if lay[1] == "t" else b.float()
    try:
        _lib.set_gemm_impl(impl)
        out = gemm(a, b, a_kmaj=lay[0] == "n", b_kmaj=lay[1] == "t",
                   out_dtype=torch.bfloat16 if lay[0] == "n" else torch.float32)
        torch.cuda.synchronize()
    finally:
        _lib.set_gemm_impl(-1)
    assert _rel(out, am @ bm) < 1e-2, _rel(out, am @ bm)
