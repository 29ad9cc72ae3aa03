"""LayerNorm backward: persistent-grid size sweep (GB/s moved) at the GPT-2 shapes.

    python bench/ln_grid.py
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.norm import layernorm_bwd, layernorm_fwd  # noqa: E402


def timeit(fn, iters=20, reps=3):
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
    import sys
    shapes = ((32736, 768), (16368, 1600))
    if len(sys.argv) > 1:  # e.g. 16320x256,65472x768
        shapes = tuple(tuple(int(v) for v in a.split("x")) for a in sys.argv[1].split(","))
    for T, D in shapes:
        x = torch.randn(T, D, device="cuda")
        g, b = torch.randn(D, device="cuda"), torch.randn(D, device="cuda")
        _, mean, rstd = layernorm_fwd(x, g, b)
        dy = torch.randn(T, D, device="cuda").bfloat16()
        dx = torch.randn(T, D, device="cuda")
        dg, db = torch.zeros(D, device="cuda"), torch.zeros(D, device="cuda")
        gout = torch.empty(T, D, device="cuda", dtype=torch.bfloat16)
        gsum = torch.zeros(D, device="cuda")
        nbytes = T * D * (4 + 2 + 4 + 4 + 2)  # x, dy, dx r/w, gout
        for blocks in (64, 128, 256, 512, 1024, 2048, 4096):
            _lib.lib().dpc_layernorm_set_bwd_blocks(blocks)
            ms = timeit(lambda: layernorm_bwd(dy, x, mean, rstd, g, dx, dg, db, gout=gout, gsum=gsum))
            print(json.dumps({"T": T, "D": D, "blocks": blocks, "us": round(ms * 1e3, 1),
                              "GBps": round(nbytes / ms / 1e6)}), flush=True)
        _lib.lib().dpc_layernorm_set_bwd_blocks(0)


if __name__ == "__main__":
    main()
