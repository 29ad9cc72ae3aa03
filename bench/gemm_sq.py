"""Square-GEMM ceiling check: our impls vs torch (hipBLASLt) at one large shape.

    python bench/gemm_sq.py --n 8192 --impls 2 10 20
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import gemm  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernels import timeit  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, nargs="+", default=[8192])
ap.add_argument("--impls", type=int, nargs="+", default=[2, 10, 20])
a = ap.parse_args()
for n in a.n:
    x = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
    w = (torch.rand(n, n, device="cuda") * 2 - 1).bfloat16()
    fl = 2.0 * n ** 3
    res = {"n": n, "torch": round(fl / timeit(lambda: x @ w.t(), 10) / 1e9)}
    for i in a.impls:
        _lib.set_gemm_impl(i)
        res[f"impl{i}"] = round(fl / timeit(lambda: gemm(x, w), 10) / 1e9)
    _lib.set_gemm_impl(-1)
    print(res, flush=True)
