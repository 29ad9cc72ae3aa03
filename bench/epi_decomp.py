"""Where the fused FFN epilogues' time goes: the same product with its epilogue built up one
piece at a time (plain -> bias -> + one stream of GELU -> + the aux stream), each variant timed
interleaved with the others in rounds on one box (median).

    python bench/epi_decomp.py [--tokens 65472] [--dim 768] [--rounds 5] [--iters 10]
                               [--only up_full ...] [--sweep 16 21 25 ...]

Cases (GPT-2 FFN, T tokens, D model dim):
  up_*   : [T, D] x [4D, D]^T forward (v9 EPI 1 when an epilogue is present: impl 26)
  dg_*   : [T, D] x [D, 4D] input gradient of the down projection (act' of the up pre-activation,
           column sums = the up-projection bias gradient: v7 EPI 8)
  dn_*   : [T, 4D] x [D, 4D]^T forward of the down projection (bias + GELU + f32 residual)
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
from distributed_pytorch_cookbook_amd.ops.gemm import ACT_GELU, gemm  # noqa: E402


def time_ms(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=64 * 1023)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", nargs="*", default=None)
    ap.add_argument("--json", default=None)
    ap.add_argument("--sweep", type=int, nargs="*", default=[],
                    help="also time up_full / dg_full / dn_full with these implementations forced")
    a = ap.parse_args()
    T, D = a.tokens, a.dim
    dev = "cuda"
    torch.manual_seed(0)

    def r(*s):
        return torch.randn(*s, device=dev).bfloat16()

    x, xu = r(T, D), r(T, 4 * D)
    w_up, w_down = r(4 * D, D), r(D, 4 * D)
    b_d, b_4d = torch.randn(D, device=dev), torch.randn(4 * D, device=dev)
    res = torch.randn(T, D, device=dev)
    out_f = torch.empty(T, D, device=dev)
    out_u = torch.empty(T, 4 * D, device=dev, dtype=torch.bfloat16)
    aux = torch.empty(T, 4 * D, device=dev, dtype=torch.bfloat16)
    aux_d = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    dz2 = r(T, D)
    colsum = torch.zeros(4 * D, device=dev)
    up_kw = dict(a_kmaj=True, b_kmaj=True, out=out_u)
    dg_kw = dict(a_kmaj=True, b_kmaj=False, out=out_u)
    dn_kw = dict(a_kmaj=True, b_kmaj=True)
    # (name, impl forced or -1 for the table's choice, fn)
    cases = [
        ("up_plain", -1, lambda: gemm(x, w_up, **up_kw)),
        ("up_bias", 26, lambda: gemm(x, w_up, bias=b_4d, **up_kw)),
        ("up_bias_gelu", 26, lambda: gemm(x, w_up, bias=b_4d, act=ACT_GELU, **up_kw)),
        ("up_bias_aux", 26, lambda: gemm(x, w_up, bias=b_4d, aux_out=aux, **up_kw)),
        ("up_full", 26, lambda: gemm(x, w_up, bias=b_4d, act=ACT_GELU, aux_out=aux, **up_kw)),
        ("up_full_tab", -1, lambda: gemm(x, w_up, bias=b_4d, act=ACT_GELU, aux_out=aux, **up_kw)),
        ("dg_plain", -1, lambda: gemm(dz2, w_down, **dg_kw)),
        ("dg_act", -1, lambda: gemm(dz2, w_down, act_bwd=ACT_GELU, aux_in=aux, **dg_kw)),
        ("dg_colsum", -1, lambda: gemm(dz2, w_down, colsum=colsum, **dg_kw)),
        ("dg_full", -1, lambda: gemm(dz2, w_down, act_bwd=ACT_GELU, aux_in=aux, colsum=colsum, **dg_kw)),
        ("dn_plain_f32", -1, lambda: gemm(xu, w_down, out=out_f, **dn_kw)),
        ("dn_bias_res", -1, lambda: gemm(xu, w_down, bias=b_d, residual=res, out=out_f, **dn_kw)),
        ("dn_full", -1, lambda: gemm(xu, w_down, bias=b_d, act=ACT_GELU, residual=res, aux_out=aux_d, out=out_f,
                                     **dn_kw)),
    ]
    for im in a.sweep:
        cases += [(f"{name}@{im}", im, fn) for name, _, fn in cases if name in ("up_full", "dg_full", "dn_full")]
    if a.only:
        cases = [c for c in cases if c[0].split("@")[0] in a.only]
    fns = {}
    for name, impl, fn in cases:
        # impl: forced implementation (-1 = table), or (impl, {lab variant key: value})
        impl, var = impl if isinstance(impl, tuple) else (impl, {})

        def run(impl=impl, fn=fn, var=var):
            _lib.set_gemm_impl(impl)
            for k in range(2):
                _lib.set_gemm_variant(k, var.get(k, -1))
            fn()
        run()
        torch.cuda.synchronize()
        fns[name] = run
    times = {k: [] for k in fns}
    for _ in range(a.rounds):
        for k, fn in fns.items():
            times[k].append(time_ms(fn, a.iters))
    _lib.set_gemm_impl(-1)
    for k in range(2):
        _lib.set_gemm_variant(k, -1)
    fl = 2.0 * T * 4 * D * D
    rows = []
    for k, v in times.items():
        ms = statistics.median(v)
        row = dict(case=k, us=round(ms * 1e3, 1), tflops=round(fl / ms / 1e9, 1), spread_us=round((max(v) - min(v)) * 1e3, 1))
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
