"""Greedy decode latency on one GPU: LM head on every position (the reference's
``utils.generate``, /root/reference/utils.py:57-65) vs the last position only vs the
KV-cache decode (one token per forward), eager and as a replayed HIP graph.

    python bench/generate.py [--model gpt2-small] [--ctx 1000] [--tokens 20]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.models.gpt import PRESETS, TransformerDecoderLM  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--ctx", type=int, default=1000)
    ap.add_argument("--tokens", type=int, default=20)
    ap.add_argument("--graph_only", action="store_true", help="only the HIP-graph KV-cache decode (profiling)")
    a = ap.parse_args()
    p = PRESETS[a.model]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    with dev:
        m = TransformerDecoderLM(p["dim"], p["head_dim"], p["heads"], p["num_layers"], 50257, 1024,
                                 activation=p["activation"])
    m.eval()
    res = {}
    for last_only in (() if a.graph_only else (False, True)):
        ids = torch.randint(0, 50257, (1, a.ctx), device=dev)
        with torch.inference_mode():
            for i in range(a.tokens + 3):
                if i == 3:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                s = ids.shape[1]
                pos = torch.arange(s, device=dev).unsqueeze(0)
                logits = m(ids, pos, last_only=True) if last_only else m(ids, pos)
                nxt = logits[0, -1].argmax().view(1, 1)
                ids = torch.cat([ids, nxt], 1)
            torch.cuda.synchronize()
        res["last_only" if last_only else "all_positions"] = (time.perf_counter() - t0) / a.tokens * 1e3
    ids = torch.randint(0, 50257, (1, a.ctx), device=dev)
    with torch.inference_mode():
        cache = m.new_kv_cache(1, a.ctx + a.tokens + 4)
        logits = m.decode(ids, torch.arange(a.ctx, device=dev).unsqueeze(0), cache)
        for i in range(0 if a.graph_only else a.tokens + 3):
            if i == 3:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            nxt = logits[0, -1].argmax().view(1, 1)
            logits = m.decode(nxt, torch.full((1, 1), cache.len, device=dev), cache)
        torch.cuda.synchronize()
    if not a.graph_only:
        res["kv_cache"] = (time.perf_counter() - t0) / a.tokens * 1e3
    ids = torch.randint(0, 50257, (1, a.ctx), device=dev)
    with torch.inference_mode():
        cache = m.new_kv_cache(1, a.ctx + a.tokens + 4)
        logits = m.decode(ids, torch.arange(a.ctx, device=dev).unsqueeze(0), cache)
        dec = m.graph_decoder(cache)
        for i in range(a.tokens + 3):
            if i == 3:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            nxt = logits[0, -1].argmax().view(1, 1)
            logits = dec.step(nxt)
        torch.cuda.synchronize()
    res["kv_cache_graph"] = (time.perf_counter() - t0) / a.tokens * 1e3
    if a.graph_only:
        print(json.dumps({"model": a.model, "ctx": a.ctx, "ms_per_token": res}))
        return
    print(json.dumps({"model": a.model, "ctx": a.ctx, "ms_per_token": res,
                      "speedup_last_only": res["all_positions"] / res["last_only"],
                      "speedup_kv_cache": res["all_positions"] / res["kv_cache"],
                      "speedup_kv_cache_graph": res["all_positions"] / res["kv_cache_graph"]}))


if __name__ == "__main__":
    main()
