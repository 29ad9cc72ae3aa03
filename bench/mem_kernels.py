"""Memory-bound kernels of the GPT-2-small DDP step at their step shapes, as HBM bytes / time
against a device-copy roofline (one read + one write of an f32 buffer).

    python bench/mem_kernels.py [--tokens 65472 --dim 768 --params 124475904] [--rounds 5]

Variants interleave in rounds inside one process (median).  On MI355X every one of them runs at
0.9-1.05x the copy roofline (profiles/r3_memk/mem_kernels.txt); an unrolled, non-temporal AdamW
variant measured the same as the shipped one (825.6 vs 828.9 us) and was dropped.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops.elementwise import bias_act_bwd  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import ACT_GELU  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.loss import cross_entropy_rows  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.norm import layernorm_bwd, layernorm_fwd  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.optim import FlatAdamW  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65472)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--vocab", type=int, default=50257)
    ap.add_argument("--params", type=int, default=124475904)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    T, D, dev = a.tokens, a.dim, "cuda"
    f32 = lambda *s: torch.randn(*s, device=dev)  # noqa: E731
    bf = lambda *s: torch.randn(*s, device=dev).bfloat16()  # noqa: E731

    x, g, b = f32(T, D), 1 + 0.1 * f32(D), 0.1 * f32(D)
    y = torch.empty(T, D, device=dev, dtype=torch.bfloat16)
    add_y, add_b, x_out = bf(T, D), f32(D), torch.empty(T, D, device=dev)
    _, mean, rstd = layernorm_fwd(x, g, b)
    dy, dx, dg, db = bf(T, D), f32(T, D), torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    gout, gsum = torch.empty(T, D, device=dev, dtype=torch.bfloat16), torch.zeros(D, device=dev)
    dyf, z, dz, dbb = f32(T, D), bf(T, D), torch.empty(T, D, device=dev, dtype=torch.bfloat16), torch.zeros(D, device=dev)
    n = a.params // 4 * 4
    p, pg = f32(n), 1e-3 * f32(n)
    shadow = torch.empty(n, device=dev, dtype=torch.bfloat16)
    opt = FlatAdamW(p, pg, shadow=shadow)
    ld = (a.vocab + 63) // 64 * 64
    logits = bf(T, ld)
    tg = torch.randint(0, a.vocab, (T,), device=dev)
    inv = torch.full((), 1.0 / T, device=dev)
    rl = torch.empty(T, device=dev)
    src, dst = f32(T, 4 * D), torch.empty(T, 4 * D, device=dev)

    E = T * D
    variants = [
        ("copy_f32", lambda: dst.copy_(src), 8 * T * 4 * D),
        ("ln_fwd", lambda: layernorm_fwd(x, g, b, out=y), 6 * E),
        ("ln_fwd_add", lambda: layernorm_fwd(x, g, b, out=y, add=(add_y, add_b, None), x_out=x_out), 12 * E),
        ("ln_bwd", lambda: layernorm_bwd(dy, x, mean, rstd, g, dx, dg, db), 14 * E),
        ("ln_bwd_gout", lambda: layernorm_bwd(dy, x, mean, rstd, g, dx, dg, db, gout=gout, gsum=gsum), 16 * E),
        ("bias_gelu_bwd", lambda: bias_act_bwd(dyf, z, ACT_GELU, dbb, out=dz), 8 * E),
        ("ce", lambda: cross_entropy_rows(logits, tg, a.vocab, inv, rl), 4 * T * ld),
        ("adamw", opt.step, 30 * n),
    ]
    for _, fn, _ in variants:
        fn()
    torch.cuda.synchronize()
    times = {v[0]: [] for v in variants}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for name, fn, _ in variants:
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            e1.synchronize()
            times[name].append(e0.elapsed_time(e1) / a.iters * 1e3)
    for name, _, nbytes in variants:
        us = statistics.median(times[name])
        print(json.dumps({"kernel": name, "us": round(us, 1), "TBps": round(nbytes / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
