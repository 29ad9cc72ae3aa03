#!/usr/bin/env python
"""Headline benchmark: GPT-2 training tokens/sec (whole node) on N MI355X GPUs.

    python bench.py [--gpus 1] [--steps 20] [--warmup 5]            # 1 GPU
    python bench.py --gpus N --steps K --warmup W                     # N GPUs (self-launch)
    torchrun --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W                        # N GPUs

Without torchrun (``WORLD_SIZE`` unset) and N > 1, this process starts the N ranks itself as a
``torch.distributed.run`` child and relays rank 0's line; under torchrun, a ``WORLD_SIZE`` that
differs from ``--gpus`` is an error (exit 2), never a silently relabelled run.

Metric and config follow BASELINE.json ("tokens/sec (node) GPT-2 training per recipe"):
default is the ``main-ddp.py`` north-star config -- GPT-2 small (untied lm_head, 163M
params), seq_len 1024, bf16 compute, data parallel over all ranks, weak scaling
(``--batch_size`` sequences per GPU).  ``--recipe fsdp|pipe|pipe_ddp`` and ``--model``
select the other north-star configs.  Random-init weights, synthetic token batches
(no network); every timed step is a full forward + backward + gradient all-reduce +
AdamW update.  W untimed warmup steps, then exactly K steps bracketed by barrier +
device synchronize; the time is the MAX over ranks; rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from distributed_pytorch_cookbook_amd.config import apply_preset, build_parser  # noqa: E402
from distributed_pytorch_cookbook_amd.parallel import comm  # noqa: E402
from distributed_pytorch_cookbook_amd.utils.metrics import mfu, train_flops_per_token  # noqa: E402

METRIC = "tokens/sec (node) GPT-2 training per recipe (DDP/FSDP/PP) at 1/2/4/8 MI355X"
# The reference publishes no numbers.  vs_baseline compares against the
# stock-PyTorch run of the reference's own default recipe (manual attention + torch.compile,
# bf16 autocast, fused AdamW) measured on one MI355X at the same per-GPU batch x 1024 tokens
# (bench/baseline_torch.py --compile; profiles/r1_stock_pytorch_baselines.jsonl), scaled
# linearly with the GPU count.
# The other recipes (round 6, profiles/r6_stock/stock.jsonl): the same reference math + compile on one
# MI355X at 64 sequences per GPU -- gradient accumulation where one 64-sequence batch of
# materialised scores does not fit (medium / large 16 x 4, XL 8 x 8: the same optimizer step).
BASELINE_TOKS_PER_GPU = {("ddp", "gpt2-small", 32, 1024): 276672.6,
                         ("ddp", "gpt2-small", 64, 1024): 300633.0,
                         ("fsdp", "gpt2-xl", 64, 1024): 32427.5,
                         ("pipe", "gpt2-medium", 64, 1024): 114526.6,
                         ("pipe_ddp", "gpt2-large", 64, 1024): 57297.5}
# Per-GPU batch (sequences) per recipe when --batch_size is not given: every recipe runs the
# reference's own default per-rank batch (--batch_size 64, main-*.py argparse).
# On one MI355X that is also the fastest measured (profiles/r2_recipes/batch_sweep_s4.txt):
# GPT-2 XL FSDP 32 / 48 / 64 -> 78.8 / 78.2 / 80.5K tok/s at 121 / 168 / 214 GiB peak, GPT-2 large
# PP x DP 32 -> 64 +3 %, GPT-2 medium pipeline 64 -> 96 -3 %.
DEFAULT_BATCH = {"ddp": 64, "fsdp": 64, "pipe": 64, "pipe_ddp": 64}


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch_ranks(n: int) -> int:
    """``python bench.py --gpus N`` without torchrun: run the same command line under
    ``torch.distributed.run`` (one fresh process per GPU, rendezvous on 127.0.0.1) as a CHILD
    process -- this process touches no GPU and never execs -- relay its output (rank 0 prints
    the JSON line) and return its exit code, non-zero if any rank failed.  The reference's
    multi-GPU recipes are torchrun-launched (``/root/reference/main-ddp.py:1-6``)."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    r = subprocess.run(cmd, env=env)
    if r.returncode != 0:
        print(f"bench.py: {n}-rank run failed with exit code {r.returncode}", file=sys.stderr)
    return r.returncode if r.returncode > 0 else (1 if r.returncode else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--recipe", default="ddp", choices=["ddp", "fsdp", "pipe", "pipe_ddp"])
    ap.add_argument("--model", default=None)
    ap.add_argument("--batch_size", type=int, default=None,
                    help="sequences per GPU (per DP replica for PP); default per recipe (DEFAULT_BATCH)")
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--bucket_mb", type=float, default=128.0)
    ap.add_argument("--reduce_dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--pp_comm_dtype", default="fp32", choices=["fp32", "bf16"],
                    help="pipe / pipe_ddp: wire dtype of the stage-boundary activations and gradients")
    ap.add_argument("--num_microbatches", type=int, default=0)
    ap.add_argument("--schedule", default=None, choices=["1f1b", "gpipe", "zb", "zb2"],
                    help="pipeline schedule; default: zb2 for pipe (the PP=8 north star: modelled stage "
                         "efficiency 0.848 against 1F1B's 0.764, profiles/r6_pp/), zb for pipe_ddp (its W "
                         "passes stay spread, so the replica all-reduce still overlaps)")
    ap.add_argument("--dp_size", type=int, default=0)
    ap.add_argument("--prefetch", type=int, default=None, help="FSDP: units all-gathered ahead")
    ap.add_argument("--no_graph", action="store_true", help="eager steps (no HIP-graph capture)")
    ap.add_argument("--graph", action="store_true",
                    help="HIP-graph capture also at N > 1 (default: only at N = 1)")
    ap.add_argument("--force_dist_path", action="store_true",
                    help="one rank on the engines' N > 1 code path over a native 1-rank RCCL communicator "
                         "(bucketed DDP store / sharded FSDP store / replica DDP store): profiles that path "
                         "on one GPU; the result is not the headline number")
    ap.add_argument("--comm", default=os.environ.get("DPC_COMM", "auto"), choices=["auto", "torch", "native", "ipc"],
                    help="collective transport (default auto: the native RCCL communicator at N > 1); ipc = the "
                         "peer-access collectives of parallel/ipc_comm.py (DDP / FSDP)")
    ap.add_argument("--json", default=None, help="also write the result line to this file")
    a = ap.parse_args()

    env_ws = os.environ.get("WORLD_SIZE")
    if env_ws is None and a.gpus > 1:
        # launched as `python bench.py --gpus N` (no torchrun): start N fresh ranks and relay
        sys.exit(_launch_ranks(a.gpus))
    if env_ws is not None and int(env_ws) != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={env_ws}; refusing to report a "
              f"{env_ws}-rank run as {a.gpus} GPUs", file=sys.stderr)
        sys.exit(2)

    batch_given = a.batch_size is not None
    if not batch_given:
        a.batch_size = DEFAULT_BATCH[a.recipe]
    if a.recipe == "pipe_ddp" and not a.dp_size:
        # the BASELINE.json hybrid: 2 pipeline stages x (N / 2) data-parallel replicas
        a.dp_size = max(1, int(os.environ.get("WORLD_SIZE", a.gpus)) // 2)
    default_model = {"ddp": "gpt2-small", "fsdp": "gpt2-xl", "pipe": "gpt2-medium",
                     "pipe_ddp": "gpt2-large"}[a.recipe]
    model_name = a.model or default_model
    rec = "pipe_ddp" if a.recipe == "pipe_ddp" else a.recipe
    argv = ["--model", model_name, "--batch_size", str(a.batch_size), "--bucket_mb", str(a.bucket_mb),
            "--reduce_dtype", a.reduce_dtype, "--synthetic_data", "--comm", a.comm]
    if a.schedule is None:
        a.schedule = "zb2" if rec == "pipe" else "zb"
    if rec in ("pipe", "pipe_ddp"):
        argv += ["--schedule", a.schedule, "--num_microbatches", str(a.num_microbatches),
                 "--pp_comm_dtype", a.pp_comm_dtype]
    if rec == "pipe_ddp" and a.dp_size:
        argv += ["--dp_size", str(a.dp_size)]
    if rec == "fsdp" and a.prefetch is not None:
        argv += ["--prefetch", str(a.prefetch)]
    # N > 1 runs eager steps unless --graph: on one MI355X the graphed and the eager step take
    # the same time at the default batch (profiles/r1_v19_eager_vs_graph: 77.2 vs 77.2 ms), and
    # a step graph with RCCL collectives inside cannot be rehearsed on a one-GPU box (RCCL
    # refuses two ranks per device), so the scaling runs take the path without the capture
    if a.no_graph or (int(os.environ.get("WORLD_SIZE", "1")) > 1 and not a.graph):
        argv += ["--disable_compile"]
    args = build_parser(rec).parse_args(argv)
    apply_preset(args)
    args.sequence_length = a.seq_len

    info = comm.init_dist(force_group=a.force_dist_path)
    from distributed_pytorch_cookbook_amd.recipes import build_engine, build_model

    vocab = 50257
    model = build_model(args, vocab, info.device)
    engine = build_engine(rec, model, info, args, force_dist=a.force_dist_path)

    # synthetic batches: a small pool of distinct random token batches per DP replica
    S = a.seq_len
    B = a.batch_size
    pp = max(1, info.world_size // max(engine.dp_world, 1))
    if not batch_given and a.recipe in ("pipe", "pipe_ddp"):
        # weak scaling for pipelines too: each pipeline replica gets pp x the per-GPU batch,
        # so every GPU still processes DEFAULT_BATCH sequences per step (2 pp micro-batches
        # of DEFAULT_BATCH / 2 sequences each, as at N = 1)
        B = a.batch_size * pp
    g = torch.Generator(device="cpu").manual_seed(1000 + engine.dp_rank)
    pool = []
    for _ in range(4):
        ids = torch.randint(0, vocab, (B, S), generator=g)
        inputs = ids[:, :-1].to(info.device)
        targets = ids[:, 1:].to(info.device)
        pos = torch.arange(S - 1, device=info.device).unsqueeze(0).expand(B, -1)
        pool.append((dict(input_ids=inputs, position_ids=pos, mask=None), targets))

    def step(i):
        b, t = pool[i % len(pool)]
        return engine.train_step(b, t)

    for i in range(a.warmup):
        step(i)
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = None
    for i in range(a.steps):
        loss = step(i)
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    if info.device.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dt_t = torch.tensor([dt], dtype=torch.float64, device=info.device)
    if info.world_size > 1 or a.force_dist_path:
        torch.distributed.all_reduce(dt_t, op=torch.distributed.ReduceOp.MAX)
    dt = float(dt_t.item())
    # the loss lives on the ranks that own the head (last pipeline stage): average those
    lt = torch.tensor([float(loss) if loss is not None else 0.0, 1.0 if loss is not None else 0.0],
                      dtype=torch.float64, device=info.device)
    if info.world_size > 1:
        torch.distributed.all_reduce(lt)
    loss_v = float(lt[0] / lt[1]) if lt[1] > 0 else float("nan")
    peak = torch.tensor([torch.cuda.max_memory_allocated(info.device) / 2**30 if info.device.type == "cuda" else 0.0],
                        dtype=torch.float64, device=info.device)
    if info.world_size > 1:
        torch.distributed.all_reduce(peak, op=torch.distributed.ReduceOp.MAX)
    tokens_per_step = B * (S - 1) * engine.dp_world
    value = tokens_per_step * a.steps / dt
    n = info.world_size
    par = {"ddp": f"dp{n}", "fsdp": f"fsdp{n}", "pipe": f"pp{n}",
           "pipe_ddp": f"pp{n // max(engine.dp_world, 1)}xdp{engine.dp_world}"}[a.recipe]
    base = BASELINE_TOKS_PER_GPU.get((a.recipe, model_name, a.batch_size, S))
    base = base * n if base else None
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "tokens/s",
        "n_gpus": n,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000 * dt / a.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(value / base, 3) if base else None),
        "dtype": "bf16",
        "data": "synthetic",
        "config": {"model": model_name, "global_batch": B * engine.dp_world, "seq_len": S,
                   "parallelism": par, "recipe": f"main-{a.recipe.replace('_', '-')}.py",
                   "tokens_per_step": tokens_per_step, "final_loss": round(loss_v, 4),
                   "peak_mem_gib": round(float(peak.item()), 1),
                   "force_dist_path": bool(a.force_dist_path),
                   "reduce_dtype": a.reduce_dtype, "pp_comm_dtype": a.pp_comm_dtype,
                   "schedule": a.schedule if a.recipe in ("pipe", "pipe_ddp") else None,
                   "comm": getattr(getattr(engine, "store", None), "tp", None).kind
                   if getattr(getattr(engine, "store", None), "tp", None) is not None else None,
                   "step_graph": getattr(getattr(engine, "_stepper", None), "graph", None) is not None,
                   "mfu_per_gpu": round(mfu(value / n, train_flops_per_token(
                       args.dim, args.heads, args.head_dim, args.num_layers, vocab, S)), 4),
                   "baseline": ("stock PyTorch reference-default recipe (manual attention + torch.compile)"
                                " per GPU x n_gpus" if base else None)},
    }
    if info.is_main:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json:
            os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
            with open(a.json, "w") as f:
                f.write(line + "\n")
    comm.cleanup_dist()


if __name__ == "__main__":
    main()
