"""Time vs K at fixed M x N (forward layout): separates per-tile fixed cost (prologue /
epilogue) from the per-k-slice main-loop cost.   python bench/gemm_kscan.py --impls 2 10 20"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import gemm  # noqa: E402

from kernels import timeit  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--impls", type=int, nargs="+", default=[2, 10, 20])
ap.add_argument("--M", type=int, default=32736)
ap.add_argument("--N", type=int, default=3072)
ap.add_argument("--Ks", type=int, nargs="+", default=[256, 768, 1536, 3072, 6144])
ap.add_argument("--epi", action="store_true", help="bias + gelu + aux_out epilogue (the up projection)")
a = ap.parse_args()
M, N = a.M, a.N
r = lambda *s: torch.randn(*s, device="cuda").bfloat16()  # noqa: E731
bias = torch.randn(N, device="cuda")
aux = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for i in a.impls:
    _lib.set_gemm_impl(i)
    row = []
    for K in a.Ks:
        A, B = r(M, K), r(N, K)
        kw = dict(bias=bias, act=2, aux_out=aux) if a.epi else {}
        ms = timeit(lambda: gemm(A, B, out=out, **kw), 10, 3)
        row.append(f"K{K}:{ms * 1e3:.0f}us/{2 * M * N * K / ms / 1e9:.0f}TF")
    print(f"impl{i} M={M} N={N} epi={a.epi}: " + " ".join(row), flush=True)
_lib.set_gemm_impl(-1)
