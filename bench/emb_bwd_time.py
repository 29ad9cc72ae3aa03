"""Embedding backward (sorted, deterministic segmented sums) at the GPT-2 small step shape:
token table (random ids over the vocabulary) and position table (positions 0..S-1 repeated per
sequence), timed with HIP events, one JSON line; run it under rocprofv3 --kernel-trace --stats
for the per-kernel split.

    python bench/emb_bwd_time.py [--N 64] [--S 1023] [--D 768] [--V 50257] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops.embedding import embedding_bwd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--S", type=int, default=1023)
    ap.add_argument("--D", type=int, default=768)
    ap.add_argument("--V", type=int, default=50257)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    T = a.N * a.S
    dout = torch.randn(T, a.D, device="cuda")
    ids = torch.randint(0, a.V, (T,), device="cuda")
    pos = torch.arange(a.S, device="cuda").repeat(a.N)
    dtok = torch.zeros(a.V, a.D, device="cuda")
    dpos = torch.zeros(1024, a.D, device="cuda")
    out = {}
    for name, kw in (("tok", dict(dtok=dtok, dpos=None)), ("pos", dict(dtok=None, dpos=dpos)),
                     ("both", dict(dtok=dtok, dpos=dpos))):
        def fn():
            embedding_bwd(dout, ids, pos, **kw)
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            fn()
        e.record()
        e.synchronize()
        out[name + "_us"] = round(s.elapsed_time(e) / a.iters * 1e3, 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
