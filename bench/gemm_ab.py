"""A/B the hand-written GEMM implementations against hipBLASLt (torch.mm) on random data.

    python bench/gemm_ab.py [--impls 20 26] [--shapes square|gpt2s|all] [--rounds 3]

Every variant of a shape is timed in interleaved rounds inside one process (HIP events over
``--iters`` back-to-back launches, median over rounds), and checked once against an f32
product of the same bf16 operands (max |err| relative to max |ref|).
Layouts: nt = A, B k-major (forward), nn = B n-major (input gradient), tn = both mn-major
(weight gradient, f32 accumulate).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import gemm  # noqa: E402


SQUARE = [("sq8k_nt", 8192, 8192, 8192, "nt"), ("sq8k_nn", 8192, 8192, 8192, "nn"),
          ("sq8k_tn", 8192, 8192, 8192, "tn"), ("sq4k_nt", 4096, 4096, 4096, "nt")]
T = 64 * 1023
GPT2S = [("qkv_fwd", T, 2304, 768, "nt"), ("out_fwd", T, 768, 768, "nt"),
         ("lm_fwd", T, 50304, 768, "nt"), ("qkv_dgrad", T, 768, 2304, "nn"),
         ("out_dgrad", T, 768, 768, "nn"), ("up_dgrad", T, 768, 3072, "nn"),
         ("lm_dgrad", T, 768, 50304, "nn"), ("up_fwd", T, 3072, 768, "nt"),
         ("down_fwd", T, 768, 3072, "nt")]
# GPT-2 XL (FSDP bench: 32 x 1023 tokens, D = 1600) plain products: forward, input and weight
# gradients
TX = 32 * 1023
XL = [("xl_qkv_fwd", TX, 4800, 1600, "nt"), ("xl_outp_fwd", TX, 1600, 1600, "nt"),
      ("xl_lm_fwd", TX, 50304, 1600, "nt"), ("xl_qkv_dgrad", TX, 1600, 4800, "nn"),
      ("xl_out_dgrad", TX, 1600, 1600, "nn"), ("xl_up_dgrad", TX, 1600, 6400, "nn"),
      ("xl_lm_dgrad", TX, 1600, 50304, "nn"), ("xl_w_qkv", 4800, 1600, TX, "tn"),
      ("xl_w_out", 1600, 1600, TX, "tn"), ("xl_w_up", 6400, 1600, TX, "tn"),
      ("xl_w_down", 1600, 6400, TX, "tn"), ("xl_w_lm", 50304, 1600, TX, "tn")]


# GPT-2 small weight gradients (tn, f32 out, split K through workspace slabs)
WGRAD = [("w_qkv", 2304, 768, T, "tn"), ("w_out", 768, 768, T, "tn"), ("w_up", 3072, 768, T, "tn"),
         ("w_down", 768, 3072, T, "tn"), ("w_lm", 50304, 768, T, "tn")]


# fused-epilogue products of the GPT-2 layers: (name, M, N, K, layout, epilogue)
#   up   = bias + gelu + aux_out (pre-activation), bf16 out          (FFN up forward)
#   down = bias + gelu + aux_out + f32 residual, f32 out             (FFN down forward, quirk act)
#   out  = bias + f32 residual, f32 out                              (attention out-proj forward)
#   dact = act'(aux_in) + bias-gradient column sums, bf16 out        (FFN input gradient)
FUSED = [("s_up_fwd", T, 3072, 768, "nt", "up"), ("s_down_fwd", T, 768, 3072, "nt", "down"),
         ("s_out_fwd", T, 768, 768, "nt", "out"), ("s_dact", T, 3072, 768, "nn", "dact"),
         ("xl_down_fwd", 32736, 1600, 6400, "nt", "down"), ("xl_up_fwd", 32736, 6400, 1600, "nt", "up"),
         ("xl_out_fwd", 32736, 1600, 1600, "nt", "out"), ("xl_dact", 32736, 6400, 1600, "nn", "dact")]


def epilogue(kind, M, N, dev="cuda"):
    kw = {}
    if kind in ("up", "down", "out"):
        kw["bias"] = torch.randn(N, device=dev)
    if kind in ("up", "down"):
        kw["act"] = 2
        kw["aux_out"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if kind in ("down", "out"):
        kw["residual"] = torch.randn(M, N, device=dev)
        kw["out_dtype"] = torch.float32
    if kind == "dact":
        kw["act_bwd"] = 2
        kw["aux_in"] = torch.randn(M, N, device=dev).bfloat16()
        kw["colsum"] = torch.zeros(N, device=dev)
    return kw


def operands(M, N, K, lay, dev="cuda"):
    r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()  # noqa: E731
    if lay == "nt":
        return r(M, K), r(N, K), dict(a_kmaj=True, b_kmaj=True), torch.bfloat16
    if lay == "nn":
        return r(M, K), r(K, N), dict(a_kmaj=True, b_kmaj=False), torch.bfloat16
    return r(K, M), r(K, N), dict(a_kmaj=False, b_kmaj=False), torch.float32


def torch_fn(A, B, lay, out):
    if lay == "nt":
        return lambda: torch.mm(A, B.t(), out=out)
    if lay == "nn":
        return lambda: torch.mm(A, B, out=out)
    return lambda: torch.ops.aten.mm.dtype_out(A.t(), B, torch.float32, out=out)


def time_ms(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def check(A, B, lay, out):
    am = A.float() if lay != "tn" else A.float().t()
    bm = B.float().t() if lay == "nt" else B.float()
    ref = am @ bm
    return float((out.float() - ref).abs().max() / ref.abs().max())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", type=int, nargs="+", default=[20, 26])
    ap.add_argument("--shapes", default="all", choices=["square", "gpt2s", "all", "fused", "xl", "wgrad"])
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    shapes = (SQUARE if a.shapes in ("square", "all") else []) + (GPT2S if a.shapes in ("gpt2s", "all") else []) + (XL if a.shapes == "xl" else []) + (WGRAD if a.shapes == "wgrad" else [])
    if a.only:
        shapes = [s for s in shapes if s[0] in a.only]
    rows = []
    if a.shapes == "fused":
        for name, M, N, K, lay, kind in FUSED:
            if a.only and name not in a.only:
                continue
            torch.manual_seed(0)
            A, B, kw, _ = operands(M, N, K, lay)
            ekw = epilogue(kind, M, N)
            times = {}
            for impl in [0] + a.impls:
                _lib.set_gemm_impl(impl if impl else -1)
                fn = lambda: gemm(A, B, **kw, **ekw)  # noqa: E731
                fn()
                torch.cuda.synchronize()
                times[f"i{impl}"] = []
            for _ in range(a.rounds):
                for impl in [0] + a.impls:
                    _lib.set_gemm_impl(impl if impl else -1)
                    times[f"i{impl}"].append(time_ms(lambda: gemm(A, B, **kw, **ekw), a.iters))
            _lib.set_gemm_impl(-1)
            fl = 2.0 * M * N * K
            row = dict(case=name, M=M, N=N, K=K, layout=lay, epilogue=kind)
            for k, v in times.items():
                ms = statistics.median(v)
                row[k] = dict(ms=round(ms, 4), tflops=round(fl / ms / 1e9, 1))
            rows.append(row)
            print(json.dumps(row), flush=True)
            del A, B, ekw
            torch.cuda.empty_cache()
        shapes = []
    for name, M, N, K, lay in shapes:
        torch.manual_seed(0)
        A, B, kw, odt = operands(M, N, K, lay)
        out = torch.empty(M, N, device="cuda", dtype=odt)
        variants = {"blas": torch_fn(A, B, lay, out),
                    # the impl the shipped table (ops/gemm_tuned.json) picks, or the policy
                    "tab": (lambda: (_lib.set_gemm_impl(-1), gemm(A, B, out=out, **kw)))}
        for impl in a.impls:
            variants[f"i{impl}"] = (lambda impl=impl: (_lib.set_gemm_impl(impl), gemm(A, B, out=out, **kw)))
        errs = {}
        for k, fn in variants.items():
            fn()
            torch.cuda.synchronize()
            if M * N * K <= 8192 ** 3:
                errs[k] = check(A, B, lay, out)
            fn()
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, fn in variants.items():
                times[k].append(time_ms(fn, a.iters))
        _lib.set_gemm_impl(-1)
        fl = 2.0 * M * N * K
        row = dict(case=name, M=M, N=N, K=K, layout=lay)
        for k in variants:
            ms = statistics.median(times[k])
            row[k] = dict(ms=round(ms, 4), tflops=round(fl / ms / 1e9, 1), err=errs.get(k))
        rows.append(row)
        print(json.dumps(row), flush=True)
        del A, B, out
        torch.cuda.empty_cache()
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
