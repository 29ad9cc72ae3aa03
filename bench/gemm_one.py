"""Run one GEMM shape repeatedly (for rocprofv3 PMC / kernel-trace collection).

    python bench/gemm_one.py --M 16368 --N 3072 --K 768 --layout nt --impl 2 --iters 50
layout: nt = forward (A k-major, B k-major), nn = dgrad (B n-major), tn = wgrad (both mn-major)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import gemm  # noqa: E402


ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=16368)
ap.add_argument("--N", type=int, default=3072)
ap.add_argument("--K", type=int, default=768)
ap.add_argument("--layout", default="nt", choices=["nt", "nn", "tn"])
ap.add_argument("--impl", type=int, default=-1)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--splits", type=int, default=0, help="force the split-K count (0: automatic)")
a = ap.parse_args()
M, N, K = a.M, a.N, a.K
r = lambda *s: torch.randn(*s, device="cuda").bfloat16()  # noqa: E731
if a.layout == "nt":
    A, B, kw = r(M, K), r(N, K), dict(a_kmaj=True, b_kmaj=True)
elif a.layout == "nn":
    A, B, kw = r(M, K), r(K, N), dict(a_kmaj=True, b_kmaj=False)
else:
    A, B, kw = r(K, M), r(K, N), dict(a_kmaj=False, b_kmaj=False)
_lib.set_gemm_impl(a.impl)
_lib.set_gemm_splits(a.splits)
out = torch.empty(M, N, device="cuda", dtype=torch.float32 if a.layout == "tn" else torch.bfloat16)
for _ in range(3):
    gemm(A, B, out=out, **kw)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(a.iters):
    gemm(A, B, out=out, **kw)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / a.iters
print(f"{a.layout} M={M} N={N} K={K} impl={a.impl} splits={a.splits}: {ms*1e3:.1f} us  {2*M*N*K/ms/1e9:.1f} TF/s")
