"""Every plain GEMM of the GPT-2 small DDP step (B = 64, S = 1024 -> T = 65472 tokens): our
default dispatch against torch.mm (hipBLASLt) on the same operands, interleaved.

    python bench/step_gemms_vs_blas.py [--T 65472] [--rounds 2]

layout nt = forward (x @ W^T), nn = input gradient (dy @ W), tn = weight gradient (dy^T @ x,
ours into an f32 accumulator as in the step, torch's output bf16).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops.gemm import gemm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--T", type=int, default=65472)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
T, D, V = a.T, 768, 50304  # (the vocabulary as the step stores it: rows padded to 64)
SHAPES = [  # name, layout, M, N, K
    ("qkv_fwd", "nt", T, 3 * D, D), ("out_fwd", "nt", T, D, D), ("head_fwd", "nt", T, V, D),
    ("qkv_dx", "nn", T, D, 3 * D), ("out_dx", "nn", T, D, D), ("up_dx", "nn", T, D, 4 * D), ("head_dx", "nn", T, D, V),
    ("qkv_dw", "tn", 3 * D, D, T), ("out_dw", "tn", D, D, T), ("up_dw", "tn", 4 * D, D, T), ("down_dw", "tn", D, 4 * D, T),
    ("head_dw", "tn", V, D, T),
]


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / a.iters * 1e3


r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
res = {}
for rnd in range(a.rounds):
    for name, lay, M, N, K in SHAPES:
        if lay == "nt":
            A, B = r(M, K), r(N, K)
            ours = lambda: gemm(A, B, a_kmaj=True, b_kmaj=True, out=C)  # noqa: E731
            blas = lambda: torch.mm(A, B.t())  # noqa: E731
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        elif lay == "nn":
            A, B = r(M, K), r(K, N)
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ours = lambda: gemm(A, B, a_kmaj=True, b_kmaj=False, out=C)  # noqa: E731
            blas = lambda: torch.mm(A, B)  # noqa: E731
        else:
            A, B = r(K, M), r(K, N)
            C = torch.zeros(M, N, device="cuda", dtype=torch.float32)
            ours = lambda: gemm(A, B, a_kmaj=False, b_kmaj=False, out=C, accumulate=True)  # noqa: E731
            blas = lambda: torch.mm(A.t(), B)  # noqa: E731
        fl = 2.0 * M * N * K
        for k, fn in (("ours", ours), ("blas", blas)):
            us = timeit(fn)
            res.setdefault((name, k), []).append(us)
        del A, B, C
        torch.cuda.empty_cache()
        print(json.dumps({"case": name, "round": rnd, "ours_us": round(res[(name, "ours")][-1], 1),
                          "blas_us": round(res[(name, "blas")][-1], 1),
                          "ours_tf": round(fl / res[(name, "ours")][-1] / 1e6), "blas_tf": round(fl / res[(name, "blas")][-1] / 1e6)}),
              flush=True)
