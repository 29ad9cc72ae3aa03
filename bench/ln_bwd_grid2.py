"""LayerNorm backward (the step's LN2 form: dy bf16, gout + column sums) over the persistent grid
size, prefetch on / off.

    python bench/ln_bwd_grid2.py [--T 65472] [--D 768]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.norm import layernorm_bwd, layernorm_fwd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--T", type=int, default=65472)
ap.add_argument("--D", type=int, default=768)
a = ap.parse_args()
T, D, dev = a.T, a.D, "cuda"
x = torch.randn(T, D, device=dev)
g, b = torch.randn(D, device=dev), torch.randn(D, device=dev)
_, mean, rstd = layernorm_fwd(x, g, b)
dy = torch.randn(T, D, device=dev).bfloat16()
dx = torch.randn(T, D, device=dev)
dg, db = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
gout = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
gsum = torch.zeros(D, device=dev)
fn = lambda: layernorm_bwd(dy, x, mean, rstd, g, dx, dg, db, gout=gout, gsum=gsum)  # noqa: E731


def timeit():
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / 20 * 1e3


for r in range(2):
    for pf in (1, 0):
        _lib.lib().dpc_layernorm_set_bwd_prefetch(pf)
        for blocks in (256, 384, 512, 768, 1024):
            _lib.lib().dpc_layernorm_set_bwd_blocks(blocks)
            print(json.dumps({"pf": pf, "blocks": blocks, "us": round(timeit(), 1)}), flush=True)
_lib.lib().dpc_layernorm_set_bwd_blocks(0)
_lib.lib().dpc_layernorm_set_bwd_prefetch(-1)
