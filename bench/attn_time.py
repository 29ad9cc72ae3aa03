"""Flash-attention forward and backward at the GPT-2 small step shape (B=64, S=1023, H=12,
hd=64 by default), each timed with HIP events over rounds (median), one JSON line.

    python bench/attn_time.py [--N 64] [--S 1023] [--H 12] [--hd 64] [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops.attention import attention_bwd, attention_fwd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--S", type=int, default=1023)
    ap.add_argument("--H", type=int, default=12)
    ap.add_argument("--hd", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    torch.manual_seed(0)
    T = a.N * a.S
    qkv = torch.randn(T, 3 * a.H * a.hd, device="cuda").bfloat16()
    o, lse = attention_fwd(qkv, a.N, a.S, a.H, a.hd)
    do = torch.randn(T, a.H * a.hd, device="cuda").bfloat16()
    dqkv = torch.empty_like(qkv)
    fns = {"fwd": lambda: attention_fwd(qkv, a.N, a.S, a.H, a.hd, out=o),
           "bwd": lambda: attention_bwd(do, qkv, o, lse, a.N, a.S, a.H, a.hd, dqkv=dqkv)}
    times = {k: [] for k in fns}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for k, f in fns.items():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                f()
            e.record()
            e.synchronize()
            times[k].append(s.elapsed_time(e) / a.iters * 1e3)
    fl = 2.0 * a.N * a.H * a.S * a.S * a.hd  # causal forward FLOPs (two products over S^2 / 2)
    row = {"shape": [a.N, a.S, a.H, a.hd]}
    for k, v in times.items():
        us = statistics.median(v)
        row[k] = {"us": round(us, 1), "pflops": round((fl if k == "fwd" else 2.5 * fl) / us / 1e9, 3)}
    print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
