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
