"""GEMM implementation sweep on the GPT-2 products WITH their fused epilogues (the ones the
model runs on dpc_gemm; the plain ones go to hipBLASLt).

    python bench/gemm_epi.py [--tokens 32736] [--impls 2 3 4 10] [--json out.json]

Cases (D = 768, T tokens): out-proj forward (bias + residual, f32 out), up-proj forward
(bias + GELU + pre-activation aux, bf16 out), down-proj forward (bias + GELU + residual, f32
out), up-proj dgrad with act' (aux in) + bias-grad column sums, and the weight gradients
(f32 accumulate, split-K).  Timed with HIP events on random data.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import ACT_GELU, gemm  # noqa: E402



def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32 * 1023)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--impls", type=int, nargs="+", default=[2, 3, 4, 10])
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    T, D = a.tokens, a.dim
    dev = "cuda"

    def r(*s):
        return torch.randn(*s, device=dev).bfloat16()

    x, xu = r(T, D), r(T, 4 * D)
    w_out, w_up, w_down = r(D, D), r(4 * D, D), r(D, 4 * D)
    b_d, b_4d = torch.randn(D, device=dev), torch.randn(4 * D, device=dev)
    res = torch.randn(T, D, device=dev)
    out_f = torch.empty(T, D, device=dev)
    out_u = torch.empty(T, 4 * D, device=dev, dtype=torch.bfloat16)
    aux = torch.empty(T, 4 * D, device=dev, dtype=torch.bfloat16)
    dz2 = r(T, D)
    colsum = torch.zeros(4 * D, device=dev)
    g_up = torch.zeros(4 * D, D, device=dev)
    g_sq = torch.zeros(D, D, device=dev)
    g_qkv = torch.zeros(3 * D, D, device=dev)
    dq = r(T, 3 * D)
    cases = [
        ("out_fwd_bias_res", T, D, D, lambda: gemm(x, w_out, bias=b_d, residual=res, out=out_f)),
        ("up_fwd_bias_gelu_aux", T, 4 * D, D,
         lambda: gemm(x, w_up, bias=b_4d, act=ACT_GELU, aux_out=aux, out=out_u)),
        ("down_fwd_bias_gelu_res", T, D, 4 * D,
         lambda: gemm(xu, w_down, bias=b_d, act=ACT_GELU, residual=res, out=out_f)),
        ("up_dgrad_actbwd_colsum", T, 4 * D, D,
         lambda: gemm(dz2, w_down, a_kmaj=True, b_kmaj=False, act_bwd=ACT_GELU, aux_in=aux, colsum=colsum,
                      out=out_u)),
        ("up_dgrad_plain", T, 4 * D, D, lambda: gemm(dz2, w_down, a_kmaj=True, b_kmaj=False, out=out_u)),
        ("up_dgrad_actbwd", T, 4 * D, D,
         lambda: gemm(dz2, w_down, a_kmaj=True, b_kmaj=False, act_bwd=ACT_GELU, aux_in=aux, out=out_u)),
        ("up_dgrad_colsum", T, 4 * D, D,
         lambda: gemm(dz2, w_down, a_kmaj=True, b_kmaj=False, colsum=colsum, out=out_u)),
        ("up_fwd_plain_kmaj", T, 4 * D, D, lambda: gemm(x, w_up, out=out_u)),
        ("up_wgrad", 4 * D, D, T, lambda: gemm(aux, x, a_kmaj=False, b_kmaj=False, out=g_up, accumulate=True)),
        ("down_wgrad", D, 4 * D, T,
         lambda: gemm(dz2, xu, a_kmaj=False, b_kmaj=False, out=g_up.view(D, 4 * D), accumulate=True)),
        ("qkv_wgrad", 3 * D, D, T, lambda: gemm(dq, x, a_kmaj=False, b_kmaj=False, out=g_qkv, accumulate=True)),
        ("out_wgrad", D, D, T, lambda: gemm(dz2, x, a_kmaj=False, b_kmaj=False, out=g_sq, accumulate=True)),
    ]
    rows = []
    for name, M, N, K, fn in cases:
        fl = 2.0 * M * N * K
        res_row = {"case": name, "M": M, "N": N, "K": K}
        _lib.set_gemm_impl(-1)
        res_row["default_tflops"] = round(fl / timeit(fn) / 1e9)
        # speed-of-light reference: the same M x N x K as a plain hipBLASLt product
        pa, pb = r(M, K), r(K, N)
        res_row["blas_plain"] = round(fl / timeit(lambda: torch.mm(pa, pb)) / 1e9)
        del pa, pb
        for impl in a.impls:
            _lib.set_gemm_impl(impl)
            try:
                res_row[f"impl{impl}"] = round(fl / timeit(fn) / 1e9)
            except Exception as exc:  # an impl that rejects the shape
                res_row[f"impl{impl}"] = str(exc)[:40]
        _lib.set_gemm_impl(-1)
        rows.append(res_row)
        print(json.dumps(res_row), flush=True)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        json.dump(rows, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
