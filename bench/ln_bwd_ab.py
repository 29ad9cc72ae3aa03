"""LayerNorm backward in the DDP step's configurations, kernel variants interleaved in one process.

    python bench/ln_bwd_ab.py [--T 65472] [--D 768] [--rounds 3]

Cases: the mid-layer LN2 (dy bf16, gout + bias colsum) and LN1 / final-norm forms (the previous
layer's FFN tail fused: gz + GELU'; dx_set for the final norm).  Variants: DPC_LN_BWD_PF 0 / 1
(one row at a time / next row's operands in flight).  Prints us and TB/s of the bytes each case
must move.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import ACT_GELU  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.norm import layernorm_bwd, layernorm_fwd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--T", type=int, default=65472)
ap.add_argument("--D", type=int, default=768)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--iters", type=int, default=20)
a = ap.parse_args()
T, D = a.T, a.D
dev = "cuda"
x = torch.randn(T, D, device=dev)
g, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
_, mean, rstd = layernorm_fwd(x, g, b)
dy = torch.randn(T, D, device=dev).bfloat16()
dx = torch.randn(T, D, device=dev)
dg, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
gout = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
gsum = torch.zeros(D, device=dev)
gz = torch.randn(T, D, device=dev).bfloat16()
cases = {
    "ln2": (lambda: layernorm_bwd(dy, x, mean, rstd, g, dx, dg, db, gout=gout, gsum=gsum), 4 + 2 + 4 + 4 + 2),
    "ln1_tail": (lambda: layernorm_bwd(dy, x, mean, rstd, g, dx, dg, db, gout=gout, gsum=gsum, gz=gz, gact=ACT_GELU),
                 4 + 2 + 4 + 4 + 2 + 2),
    "final_set": (lambda: layernorm_bwd(dy, x, mean, rstd, g, dx, dg, db, gout=gout, gsum=gsum, gz=gz, gact=ACT_GELU,
                                        dx_set=True), 4 + 2 + 4 + 2 + 2),
}


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


# the forward forms: LN1 (plain) and LN2 (fused residual add of the attention projection + bias)
yb = torch.randn(T, D, device=dev).bfloat16()
bias = torch.randn(D, device=dev)
xo = torch.empty(T, D, device=dev)
fwd = {
    "fwd_ln1": (lambda: layernorm_fwd(x, g, b), 4 + 2),
    "fwd_ln2_add": (lambda: layernorm_fwd(x, g, b, add=(yb, bias, None), x_out=xo), 4 + 2 + 4 + 2),
}
try:
    fwd["fwd_ln2_add"][0]()
except TypeError:  # (a tree whose layernorm_fwd has other keywords)
    fwd.pop("fwd_ln2_add")
for r in range(a.rounds):
    for name, (fn, bpe) in fwd.items():
        us = timeit(fn)
        print(json.dumps({"case": name, "us": round(us, 1), "TBps": round(T * D * bpe / us / 1e6, 2)}), flush=True)

res = {}
for r in range(a.rounds):
    for pf in (0, 1):
        _lib.lib().dpc_layernorm_set_bwd_prefetch(pf)
        for name, (fn, bpe) in cases.items():
            us = timeit(fn)
            res.setdefault((name, pf), []).append(us)
for (name, pf), v in sorted(res.items()):
    bpe = cases[name][1]
    best = min(v)
    print(json.dumps({"case": name, "pf": pf, "us": [round(u, 1) for u in v], "best_TBps": round(T * D * bpe / best / 1e6, 2)}))
_lib.lib().dpc_layernorm_set_bwd_prefetch(-1)
