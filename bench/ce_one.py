"""Fused cross-entropy (loss + argmax + in-place dlogits) at the GPT-2 head shape, A/B over
the kernel modes of csrc/misc.hip (0 register-resident rows, 3 the round-4 form of it, 1 / 2 streaming with 1 / 4 chunks
in flight per thread).

    python bench/ce_one.py [--tokens 65472]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.loss import cross_entropy_rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65472)
    ap.add_argument("--vocab", type=int, default=50257)
    a = ap.parse_args()
    T, V = a.tokens, a.vocab
    ld = (V + 63) // 64 * 64
    logits = torch.randn(T, ld, device="cuda").bfloat16()
    tg = torch.randint(0, V, (T,), device="cuda")
    inv = torch.full((), 1.0 / T, device="cuda")
    rl = torch.empty(T, device="cuda")
    for mode in (0, 3, 1, 0, 3, 1):
        _lib.lib().dpc_ce_set_mode(mode)
        cross_entropy_rows(logits, tg, V, inv, rl)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            cross_entropy_rows(logits, tg, V, inv, rl)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / 10
        print(json.dumps({"mode": mode, "us": round(ms * 1e3, 1),
                          "TBps_rw": round(2 * T * ld * 2 / ms / 1e9, 2)}), flush=True)
    _lib.lib().dpc_ce_set_mode(0)
    # the memory roofline of the same traffic: a device copy of the logits (one read, one write)
    dst = torch.empty_like(logits)
    for _ in range(2):
        dst.copy_(logits)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            dst.copy_(logits)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / 10
        print(json.dumps({"mode": "copy", "us": round(ms * 1e3, 1),
                          "TBps_rw": round(2 * T * ld * 2 / ms / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
