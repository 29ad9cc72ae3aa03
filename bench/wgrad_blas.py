"""Weight-gradient products dW += dY^T X (f32 accumulate): dpc_gemm (hand-written, split-K)
vs hipBLASLt through ``aten.addmm.dtype_out`` (beta = 1 into the f32 gradient buffer).

    python bench/wgrad_blas.py [--tokens 16368] [--dims 768 1600]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops.gemm import gemm  # noqa: E402



def timeit(fn, iters=10, reps=3):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=16368)
    ap.add_argument("--dims", type=int, nargs="+", default=[768, 1024, 1280, 1600])
    a = ap.parse_args()
    T = a.tokens
    for D in a.dims:
        for name, N, K in (("qkv", 3 * D, D), ("out", D, D), ("up", 4 * D, D), ("down", D, 4 * D),
                           ("head", 50257, D)):
            dy = torch.randn(T, N, device="cuda").bfloat16()
            x = torch.randn(T, K, device="cuda").bfloat16()
            g1 = torch.zeros(N, K, device="cuda")
            g2 = torch.zeros(N, K, device="cuda")
            f_ours = lambda: gemm(dy, x, a_kmaj=False, b_kmaj=False, out=g1, accumulate=True)  # noqa: E731
            f_blas = lambda: torch.ops.aten.addmm.dtype_out(g2, dy.t(), x, torch.float32,  # noqa: E731
                                                            beta=1, alpha=1, out=g2)
            g1.zero_(); g2.zero_()
            f_ours(); f_blas()
            err = ((g1 - g2).norm() / g2.norm()).item()
            fl = 2.0 * N * K * T
            r = {"D": D, "case": name, "M": N, "N": K, "K": T, "rel_err": round(err, 6),
                 "dpc_tflops": round(fl / timeit(f_ours) / 1e9), "blas_tflops": round(fl / timeit(f_blas) / 1e9)}
            print(json.dumps(r), flush=True)
            del dy, x, g1, g2


if __name__ == "__main__":
    main()
