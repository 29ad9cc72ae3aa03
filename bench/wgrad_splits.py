"""Weight-gradient GEMMs (mn-major x mn-major, K = tokens) swept over impl x split-K count.

    python bench/wgrad_splits.py [--impls 2 4 11] [--splits 1 2 4 8]
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
ap.add_argument("--impls", type=int, nargs="+", default=[2, 4, 11])
ap.add_argument("--splits", type=int, nargs="+", default=[0, 1, 2, 4, 8, 16])
ap.add_argument("--T", type=int, default=32736)
ap.add_argument("--xcd", type=int, nargs="+", default=[0])
ap.add_argument("--vocab", type=int, default=50304)
a = ap.parse_args()
T = a.T
r = lambda *s: torch.randn(*s, device="cuda").bfloat16()  # noqa: E731
for M, N in [(2304, 768), (3072, 768), (768, 3072), (768, 768), (a.vocab, 768)]:
    fl = 2.0 * M * N * T
    out = torch.zeros(M, N, device="cuda")
    A, B = r(T, (M + 7) // 8 * 8)[:, :M], r(T, N)
    for x in a.xcd:
        _lib.set_gemm_xcd_split(x)
        for i in a.impls:
            _lib.set_gemm_impl(i)
            res = {}
            for sp in a.splits:
                _lib.set_gemm_splits(sp)
                res[sp] = round(fl / timeit(lambda: gemm(A, B, a_kmaj=False, b_kmaj=False, out=out,
                                                         accumulate=True), 10, 3) / 1e9)
            print(f"M={M} N={N} K={T} impl{i} xcd{x}: " + " ".join(f"s{k}:{v}" for k, v in res.items()),
                  flush=True)
    _lib.set_gemm_splits(0)
    _lib.set_gemm_impl(-1)
    _lib.set_gemm_xcd_split(0)
