"""Resident-CU reserve of the persistent GEMMs (SURVEY.md §5.8 rule 4), on one MI355X.

An RCCL collective in flight keeps a few small workgroups resident (one per channel).  A
persistent GEMM sized to every CU then finds those CUs busy: their workgroups -- and their
whole share of the tiles -- wait until the collective ends.  Here an occupier kernel
(``dpc_occupy``: ``--occ`` workgroups spinning ``--occ_ms``) stands in for the collective on a
high-priority side stream, launched just before each GEMM; the GEMM's time is measured on the
compute stream with the reserve 0 and R.

    python bench/cu_reserve.py [--occ 16] [--reserve 16 32] [--occ_ms 2]
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

T = 64 * 1023
SHAPES = [("qkv_fwd", T, 2304, 768, "nt"), ("up_dgrad", T, 768, 3072, "nn"),
          ("w_qkv", 2304, 768, T, "tn"), ("sq8k", 8192, 8192, 8192, "nt")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--occ", type=int, nargs="+", default=[0, 8, 16])
    ap.add_argument("--reserve", type=int, nargs="+", default=[0, 16])
    ap.add_argument("--occ_ms", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    side = torch.cuda.Stream(priority=-1)
    cur = torch.cuda.current_stream()
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    for name, M, N, K, lay in SHAPES:
        r = lambda *s: (torch.rand(*s, device="cuda") * 2 - 1).bfloat16()  # noqa: E731
        if lay == "nt":
            A, B, kw = r(M, K), r(N, K), {}
        elif lay == "nn":
            A, B, kw = r(M, K), r(K, N), dict(b_kmaj=False)
        else:
            A, B, kw = r(K, M), r(K, N), dict(a_kmaj=False, b_kmaj=False, out_dtype=torch.float32)
        row = dict(case=name, M=M, N=N, K=K, layout=lay, occ_ms=a.occ_ms)
        for occ in a.occ:
            for res in a.reserve:
                _lib.set_cu_reserve(res)
                ts = []
                for rep in range(a.reps + 1):
                    torch.cuda.synchronize()
                    if occ:
                        side.wait_stream(cur)
                        _lib.occupy(occ, int(a.occ_ms * 1e6), sink, side)
                        torch.cuda._sleep(20000)  # let the occupier be dispatched first
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    gemm(A, B, **kw)
                    e.record()
                    torch.cuda.synchronize()
                    if rep:
                        ts.append(s.elapsed_time(e))
                row[f"occ{occ}_res{res}_ms"] = round(statistics.median(ts), 4)
        _lib.set_cu_reserve(0)
        print(json.dumps(row), flush=True)
        del A, B
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
