"""Re-time the GEMM implementations for the table entries whose signature matches a pattern, and
optionally write the winners into ``ops/gemm_tuned.json``.

    python bench/retune_keys.py --match ':02:c$' [--impls 16 22 24 25] [--write out.json]

A signature (ops/gemm.py:_sig) is ``MxNxK:<a><b>:<f|h>:<act><act_bwd>:<flags>`` with layouts k / m
(k-major / mn-major) and flags b(ias) x (aux_out) r(esidual) c(olsum) a(ccumulate); each entry is
rebuilt from it on random data and timed (min of 3 x 5 calls) for the table's current choice and
every listed implementation, each reached through the table entry (0 = the dispatcher policy).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops import gemm as G  # noqa: E402


def build(key: str, dev="cuda"):
    mnk, lay, out, acts, flags = key.split(":")
    M, N, K = (int(v) for v in mnk.split("x"))
    a_kmaj, b_kmaj = lay[0] == "k", lay[1] == "k"
    act, act_bwd = int(acts[0]), int(acts[1])
    def r(rows, cols):  # rows padded to a multiple of 8 elements, as the model stores operands
        buf = torch.randn(rows, (cols + 7) // 8 * 8, device=dev).bfloat16()
        return buf[:, :cols]

    a = r(M, K) if a_kmaj else r(K, M)
    b = r(N, K) if b_kmaj else r(K, N)
    o = torch.empty(M, N, device=dev, dtype=torch.float32 if out == "f" else torch.bfloat16)
    kw = dict(a_kmaj=a_kmaj, b_kmaj=b_kmaj, out=o, act=act, act_bwd=act_bwd)
    if "b" in flags:
        kw["bias"] = torch.randn(N, device=dev)
    if "x" in flags:
        kw["aux_out"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if "r" in flags:
        kw["residual"] = torch.randn(M, N, device=dev)
    if "c" in flags:
        kw["colsum"] = torch.zeros(N, device=dev)
    if "a" in flags:
        kw["accumulate"] = True
    if act_bwd:
        kw["aux_in"] = r(M, N)
    return lambda: G.gemm(a, b, **kw), 2.0 * M * N * K


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / 5)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--match", required=True)
    ap.add_argument("--impls", type=int, nargs="+", default=[16, 22, 24, 25])
    ap.add_argument("--write", default=None, help="write the updated table here")
    a = ap.parse_args()
    path = os.path.join(os.path.dirname(G.__file__), "gemm_tuned.json")
    table = json.load(open(path))
    keys = [k for k in table["impl"] if re.search(a.match, k)]
    changed = 0
    for key in keys:
        try:
            fn, fl = build(key)
            fn()
        except (RuntimeError, ValueError) as exc:
            print(json.dumps({"key": key, "skipped": str(exc)[:80]}), flush=True)
            continue
        cur = table["impl"][key]
        times = {}
        for impl in dict.fromkeys([cur] + a.impls):
            # the candidate goes through the table entry, exactly as a training step reaches the
            # dispatcher: 0 = the dispatcher's own policy ("auto"), not a forced impl 0 (which
            # set_gemm_impl would turn into the v1 register-staged kernel)
            G._table[key] = impl
            G._near_cache.clear()
            try:
                times[impl] = timeit(fn)
            except RuntimeError:
                pass
            finally:
                G._table[key] = cur
        best = min(times, key=times.get)
        row = {"key": key, "table": cur, "best": best,
               "tflops": {str(k): round(fl / v / 1e9) for k, v in times.items()}}
        # a change only when it is clearly faster (> 2 %): same-shape reruns vary by ~1 %
        if best != cur and times[best] < 0.98 * times[cur]:
            table["impl"][key] = best
            changed += 1
            row["changed"] = True
        print(json.dumps(row), flush=True)
        torch.cuda.empty_cache()
    print(json.dumps({"entries": len(keys), "changed": changed}), flush=True)
    if a.write:
        os.makedirs(os.path.dirname(a.write) or ".", exist_ok=True)
        json.dump(table, open(a.write, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
