"""Kernel microbenchmarks on the GPT-2 training shapes (HIP kernels vs stock torch ops).

    python bench/kernels.py [--tokens 16368] [--json gpurun_out/kernels.json]

Each case is timed with HIP events over `--iters` back-to-back launches after warmup,
on random data (zero-filled operands inflate MFMA clocks).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_cookbook_amd.ops.attention import attention_bwd, attention_fwd  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import gemm  # noqa: E402



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
    ap.add_argument("--tokens", type=int, default=16 * 1023)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--json", type=str, default=None)
    ap.add_argument("--impls", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--gemm_only", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    T, D, V = a.tokens, a.dim, a.vocab
    Vp = (V + 63) // 64 * 64
    rows = []

    def rnd(*s):
        return torch.randn(*s, device=dev).bfloat16()

    cases = [
        ("qkv_fwd", T, 3 * D, D), ("out_fwd", T, D, D), ("up_fwd", T, 4 * D, D),
        ("down_fwd", T, D, 4 * D), ("lm_head_fwd", T, Vp, D),
    ]
    from distributed_pytorch_cookbook_amd.ops import _lib

    def ours_impls(fn):
        res = {}
        for impl in a.impls:
            _lib.set_gemm_impl(impl)
            res[impl] = timeit(fn, a.iters)
        _lib.set_gemm_impl(-1)
        return res

    def add(name, M, N, K, fn, ref_fn):
        fl = 2 * M * N * K
        t = ours_impls(fn)
        ref = timeit(ref_fn, a.iters)
        best = min(t.values())
        r = dict(case=name, M=M, N=N, K=K, ours_ms=best, torch_ms=ref,
                 ours_tflops=fl / best / 1e9, torch_tflops=fl / ref / 1e9)
        for impl, v in t.items():
            r[f"impl{impl}_tflops"] = fl / v / 1e9
        rows.append(r)

    for name, M, N, K in cases:
        x, w = rnd(M, K), rnd(N, K)
        add(name, M, N, K, lambda: gemm(x, w), lambda: x @ w.t())
    # dgrad (B n-major) and wgrad (both mn-major) shapes
    for name, M, N, K in [("up_dgrad", T, D, 4 * D), ("qkv_dgrad", T, D, 3 * D), ("lm_dgrad", T, D, Vp)]:
        dy, w = rnd(M, K), rnd(K, N)
        add(name, M, N, K, lambda: gemm(dy, w, a_kmaj=True, b_kmaj=False), lambda: dy @ w)
    for name, M, N, K in [("up_wgrad", 4 * D, D, T), ("qkv_wgrad", 3 * D, D, T), ("lm_wgrad", V, D, T)]:
        dy = rnd(K, (M + 7) // 8 * 8)[:, :M]
        x = rnd(K, N)
        out = torch.zeros(M, N, device=dev)
        add(name, M, N, K, lambda: gemm(dy, x, a_kmaj=False, b_kmaj=False, out=out, accumulate=True),
            lambda: out.add_(dy.t() @ x))
    if a.gemm_only:
        for r in rows:
            print(json.dumps(r))
        return
    # attention (GPT-2 small: H=12, hd=64, S=1023)
    S, H, hd = 1023, 12, 64
    N = max(1, T // S)
    qkv = rnd(N * S, 3 * H * hd)
    o, lse = attention_fwd(qkv, N, S, H, hd)
    do = rnd(N * S, H * hd)
    f_fwd = timeit(lambda: attention_fwd(qkv, N, S, H, hd), a.iters)
    f_bwd = timeit(lambda: attention_bwd(do, qkv, o, lse, N, S, H, hd), a.iters)
    q = rnd(N, H, S, hd)
    k = rnd(N, H, S, hd)
    v = rnd(N, H, S, hd)
    sd_fwd = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True), a.iters)
    qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k, v))
    oo = torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=True)
    g = torch.randn_like(oo)
    sd_bwd = timeit(lambda: torch.autograd.grad(oo, (qq, kk, vv), g, retain_graph=True), a.iters)
    fl = 4 * N * H * S * S * hd / 2  # causal
    rows.append(dict(case="attn_fwd", N=N, S=S, H=H, ours_ms=f_fwd, torch_ms=sd_fwd,
                     ours_tflops=fl / f_fwd / 1e9, torch_tflops=fl / sd_fwd / 1e9))
    rows.append(dict(case="attn_bwd", N=N, S=S, H=H, ours_ms=f_bwd, torch_ms=sd_bwd,
                     ours_tflops=2.5 * fl / f_bwd / 1e9, torch_tflops=2.5 * fl / sd_bwd / 1e9))
    for r in rows:
        print(json.dumps(r))
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
