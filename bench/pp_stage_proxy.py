"""One-GPU proxy of a pipeline stage of the north-star pipeline configs.

    python bench/pp_stage_proxy.py [--model gpt2-medium --pp 8 --micro 32 --mb 16] [--graph]

Runs the decoder layers of ONE stage of the ``--pp``-way partition (``parallel/pipeline.py:
partition``, the bottleneck stage -- the most expensive group without the embeddings or the
head) through the engine's own pieces: a ``LocalStore`` over the stage's units, ``run_layers``
forward / autograd backward per micro-batch in the exact 1F1B order of that stage
(``schedule_1f1b``), the boundary tensors replaced by local buffers (f32 ``[mb * S, D]`` as
``--pp_comm_dtype fp32`` carries them, or bf16), then one fused AdamW step.  Reports per-token
time against the same layers run as ONE micro-batch of ``--full`` sequences (the pp1 step shape),
so the difference is what the micro-batching itself costs (launches, small-M GEMM tiles,
per-micro-batch allocations), eager and as a replayed HIP graph.  ``--schedule zb`` runs the
zero-bubble order (B / W split, deferred weight gradients); the per-op costs it measures feed the
pipeline simulation (``parallel/pipeline.py:simulate_orders``) for the modelled bubble and stage
efficiency of both schedules.

Reference: ``/root/reference/main-pipe.py:78-83`` (Pipe with chunks = stages).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.config import PRESETS  # noqa: E402
from distributed_pytorch_cookbook_amd.models.fused import defer_weight_grads, run_layers  # noqa: E402
from distributed_pytorch_cookbook_amd.models.gpt import TransformerDecoderLM  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.optim import FlatAdamW  # noqa: E402
from distributed_pytorch_cookbook_amd.parallel.pipeline import (bubble_factor, partition, schedule_1f1b,  # noqa: E402
                                                                schedule_zb, stage_costs, unit_costs)
from distributed_pytorch_cookbook_amd.parallel.store import LocalStore  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--pp", type=int, default=8)
    ap.add_argument("--stage", type=int, default=-1, help="-1: the most expensive middle stage")
    ap.add_argument("--micro", type=int, default=32, help="micro-batches per step")
    ap.add_argument("--mb", type=int, default=16, help="sequences per micro-batch")
    ap.add_argument("--full", type=int, default=64, help="sequences of the one-micro-batch reference")
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--wire", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--graph", action="store_true", help="also time the step as a replayed HIP graph")
    ap.add_argument("--only", default="both", choices=["both", "micro", "full"],
                    help="run one of the two steps (a kernel profile of each on its own)")
    ap.add_argument("--schedule", default="1f1b", choices=["1f1b", "zb", "zb2"],
                    help="zb: the zero-bubble order (B / W split, parallel/pipeline.py:schedule_zb)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda" if torch.cuda.is_available() else "cpu")
    cfg = PRESETS[a.model]
    S = a.seq_len
    torch.manual_seed(0)
    with torch.device("meta"):
        model = TransformerDecoderLM(dim=cfg["dim"], head_dim=cfg["head_dim"], heads=cfg["heads"],
                                     num_layers=cfg["num_layers"], vocab_size=50257, max_position_embeddings=S,
                                     activation=cfg.get("activation", "gelu"))
    groups = partition(unit_costs(model, S), a.pp)
    costs = unit_costs(model, S)
    stage = a.stage
    if stage < 0:
        mids = [s for s in range(a.pp) if 0 not in groups[s] and model.num_layers + 1 not in groups[s]] or list(range(a.pp))
        stage = max(mids, key=lambda s: sum(costs[u] for u in groups[s]))
    # the stage's decoder layers (a pp2 stage also holds the embeddings or the head: those stay
    # unmaterialised, the proxy times the layers)
    units = [u for u in groups[stage] if 1 <= u <= model.num_layers]
    layers = [model.decoder.layers[u - 1] for u in units]
    # materialise only the stage's parameters (the others stay on the meta device)
    for li in layers:
        li.to_empty(device=dev)
        for p in li.parameters():
            torch.nn.init.normal_(p, std=0.02)
    store = LocalStore(model, dev, units=units)
    opt = FlatAdamW(store.master, store.grads, lr=1e-4, shadow=store.shadow)
    D = model.dim
    wdt = torch.float32 if a.wire == "fp32" else torch.bfloat16

    def make_step(n_micro, mb):
        T = mb * (S - 1)
        xs = [torch.randn(T, D, device=dev).to(wdt) for _ in range(n_micro)]
        gs = [torch.randn(T, D, device=dev).to(wdt) * 1e-3 for _ in range(n_micro)]
        zb = a.schedule in ("zb", "zb2") and n_micro > 1
        if zb:
            order = schedule_zb(n_micro, stage, a.pp, costs=stage_costs(model, S, groups),
                                mem=2 if a.schedule == "zb2" else 1)
        else:
            order = schedule_1f1b(n_micro, stage if n_micro > 1 else 0, a.pp if n_micro > 1 else 1)
        store.accum_steps = n_micro

        def body(ev=None):
            store.zero_grad()
            live, wq = {}, {}
            for kind, m in order:
                if ev is not None:
                    ev.append((kind, torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                    ev[-1][1].record()
                if kind == "F":
                    x = xs[m].float().requires_grad_(True)  # the received boundary tensor
                    y = run_layers(model, store, x, None, mb, S - 1, layers, True)
                    live[m] = (x, y.to(wdt))  # the tensor that would be sent on
                elif kind == "B":
                    x, y = live.pop(m)
                    if zb:
                        with defer_weight_grads(wq.setdefault(m, [])):
                            torch.autograd.backward(y, gs[m])
                    else:
                        torch.autograd.backward(y, gs[m])
                    _ = x.grad.to(wdt)  # the gradient that would be sent back
                else:
                    for fn in wq.pop(m):
                        fn()
                if ev is not None:
                    ev[-1][2].record()
            opt.step(grad_scale=1.0)
        return body, n_micro * T

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def timed(body, graph):
        fn = body
        if graph:
            for _ in range(2):
                body()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                body()
            fn = g.replay
        for _ in range(a.warmup):
            fn()
        sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        sync()
        return (time.perf_counter() - t0) / a.steps

    out = {"model": a.model, "pp": a.pp, "stage": stage, "units": units, "layers": len(layers),
           "micro": a.micro, "mb": a.mb, "full": a.full, "wire": a.wire,
           "boundary_mb_per_micro": round(a.mb * (S - 1) * D * (4 if a.wire == "fp32" else 2) / 2**20, 1)}
    steps = []
    if a.only in ("both", "micro"):
        steps.append(("micro",) + make_step(a.micro, a.mb))
    if a.only in ("both", "full"):
        steps.append(("full",) + make_step(1, a.full))
    for name, body, tok in steps:
        for graph in ([False, True] if a.graph else [False]):
            dt = timed(body, graph)
            key = f"{name}_{'graph' if graph else 'eager'}"
            out[key + "_ms"] = round(dt * 1e3, 3)
            out[key + "_us_per_ktok"] = round(dt * 1e6 / tok * 1000, 3)
    ref = out.get("full_eager_us_per_ktok")
    for k in list(out):
        if ref and k.endswith("_us_per_ktok") and k != "full_eager_us_per_ktok":
            out[k.replace("_us_per_ktok", "_vs_full")] = round(out[k] / ref, 3)
    # per-op costs of the micro-batched step (one more eager step, events around every op) and the
    # modelled pipeline: bubble = simulated step time / busiest stage's work (every stage costed as
    # this one), 1F1B (B + W as one backward) against the zero-bubble order; efficiency = 1 / (tax
    # x bubble) with tax = the micro-batched step's per-token time over the one-batch step's
    if a.only in ("both", "micro") and dev.type == "cuda":
        body = steps[0][1]
        ev = []
        body(ev)
        torch.cuda.synchronize()
        tot = {"F": 0.0, "B": 0.0, "W": 0.0}
        for kind, e0, e1 in ev:
            tot[kind] += e0.elapsed_time(e1)
        cF, cB, cW = (tot[k] / a.micro for k in "FBW")
        if a.schedule == "1f1b":  # (1F1B's B holds its W: split by the cost model's share)
            sc = stage_costs(model, S, groups)[stage]
            cW = cB * sc[2] / (sc[1] + sc[2])
            cB -= cW
        out["op_ms"] = {"F": round(cF, 3), "B": round(cB, 3), "W": round(cW, 3)}
        costs = [(cF, cB, cW)] * a.pp
        tax = out.get("micro_eager_vs_full")
        for sch in ("1f1b", "zb", "zb2"):
            bf = bubble_factor(a.micro, costs, sch)
            out["bubble_" + sch] = round(bf, 3)
            if tax:
                out["eff_" + sch] = round(1.0 / (tax * bf), 3)
    line = json.dumps(out)
    print(line, flush=True)
    if a.json:
        with open(a.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
