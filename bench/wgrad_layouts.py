"""Weight-gradient shapes (small M x N, K = tokens) in all three operand layouts.

    python bench/wgrad_layouts.py --impls 2 4 10
Separates the cost of the mn-major (transposed-read) layout from the small-output /
long-K regime itself.
"""
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
ap.add_argument("--impls", type=int, nargs="+", default=[2, 4, 10])
ap.add_argument("--T", type=int, default=32736)
ap.add_argument("--layouts", nargs="+", default=["nt", "nn", "tn"])
ap.add_argument("--xcd", action="store_true", help="XCD-aligned split-K mapping")
a = ap.parse_args()
_lib.set_gemm_xcd_split(a.xcd)
T = a.T
r = lambda *s: torch.randn(*s, device="cuda").bfloat16()  # noqa: E731
for M, N in [(768, 3072), (3072, 768), (2304, 768), (768, 768)]:
    fl = 2.0 * M * N * T
    out = torch.zeros(M, N, device="cuda")
    for lay in a.layouts:
        if lay == "nt":
            A, B, kw = r(M, T), r(N, T), dict(a_kmaj=True, b_kmaj=True)
        elif lay == "nn":
            A, B, kw = r(M, T), r(T, N), dict(a_kmaj=True, b_kmaj=False)
        else:
            A, B, kw = r(T, M), r(T, N), dict(a_kmaj=False, b_kmaj=False)
        res = {}
        for i in a.impls:
            _lib.set_gemm_impl(i)
            res[i] = round(fl / timeit(lambda: gemm(A, B, out=out, accumulate=True, **kw), 10) / 1e9)
        _lib.set_gemm_impl(-1)
        print(f"M={M} N={N} K={T} {lay}: " + " ".join(f"impl{i}:{v}" for i, v in res.items()), flush=True)
