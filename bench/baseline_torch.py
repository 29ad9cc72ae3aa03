#!/usr/bin/env python
"""Stock-PyTorch-ROCm equivalent of the reference recipe (the comparison baseline).

Reference semantics with the crash bugs fixed: the reference model math in plain torch
modules (manual attention with a materialised [N,H,S,S] score tensor, as
``/root/reference/models/gpt.py:68-105``), ``torch.autocast(bf16)``, ``F.cross_entropy``,
``torch.optim.AdamW`` (fused), torch DDP for N > 1; ``--compile`` adds the reference's
default ``torch.compile`` (Inductor/Triton), ``--scaler`` its GradScaler.  ``--sdpa`` swaps the manual attention for
``F.scaled_dot_product_attention`` (a stronger stock baseline).

    python bench/baseline_torch.py --steps 10 --warmup 3 [--model gpt2-small] [--sdpa]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_pytorch_cookbook_amd.models import gpt as G  # noqa: E402
from distributed_pytorch_cookbook_amd.parallel import comm  # noqa: E402


def sdpa_forward(self, x, mask=None):
    N, S, _ = x.shape
    q = self.to_q(x).view(N, S, self.heads, self.head_dim).transpose(1, 2)
    k = self.to_k(x).view(N, S, self.heads, self.head_dim).transpose(1, 2)
    v = self.to_v(x).view(N, S, self.heads, self.head_dim).transpose(1, 2)
    o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
    return self.dropout(self.to_out(o.transpose(1, 2).reshape(N, S, -1)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch_size", type=int, default=16)
    ap.add_argument("--seq_len", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sdpa", action="store_true")
    ap.add_argument("--compile", action="store_true",
                    help="torch.compile the forward (the reference's default: Inductor/Triton)")
    ap.add_argument("--scaler", action="store_true",
                    help="GradScaler around backward/step as the reference recipes do")
    ap.add_argument("--accum", type=int, default=1,
                    help="micro-batches of --batch_size per optimizer step (gradient accumulation: the "
                         "same 64 sequences per step when the manual-attention scores of one 64-sequence "
                         "batch do not fit, e.g. GPT-2 XL)")
    ap.add_argument("--fsdp", action="store_true",
                    help="wrap in torch FSDP (FULL_SHARD, per-block auto wrap) as main-fsdp.py intends")
    a = ap.parse_args()
    info = comm.init_dist()
    dev = info.device
    p = G.PRESETS[a.model]
    if a.sdpa:
        G.SelfAttention.forward = sdpa_forward
    torch.manual_seed(0)
    with torch.device(dev):
        model = G.TransformerDecoderLM(p["dim"], p["head_dim"], p["heads"], p["num_layers"], 50257,
                                       a.seq_len, activation=p["activation"])
    fwd_model = model
    if a.fsdp:
        import functools

        import torch.distributed as dist
        from torch.distributed.fsdp import FullyShardedDataParallel as FSDP
        from torch.distributed.fsdp.wrap import size_based_auto_wrap_policy

        if not dist.is_initialized():  # (one rank: a one-member process group for FSDP)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29533")
            dist.init_process_group("nccl", rank=0, world_size=1)

        class WrapF(torch.nn.Module):
            def __init__(self, m):
                super().__init__()
                self.m = m

            def forward(self, ids, pos):
                return self.m.reference_forward(ids, pos)

        # reference main-fsdp.py:60-69 (size-based auto wrap, FULL_SHARD), with torch 2.10's kwargs
        fwd_model = FSDP(WrapF(model), device_id=dev,
                         auto_wrap_policy=functools.partial(size_based_auto_wrap_policy, min_num_params=10**6))
        model_params = fwd_model.parameters()
        call = lambda ids, pos: fwd_model(ids, pos)  # noqa: E731
    elif info.world_size > 1:
        from torch.nn.parallel import DistributedDataParallel as DDP

        class Wrap(torch.nn.Module):
            def __init__(self, m):
                super().__init__()
                self.m = m

            def forward(self, ids, pos):
                return self.m.reference_forward(ids, pos)

        fwd_model = DDP(Wrap(model), device_ids=[dev])
        call = lambda ids, pos: fwd_model(ids, pos)  # noqa: E731
    else:
        call = lambda ids, pos: model.reference_forward(ids, pos)  # noqa: E731
    if not a.fsdp:
        model_params = model.parameters()
    if a.compile:
        call = torch.compile(call)
    opt = torch.optim.AdamW(model_params, lr=1e-4, fused=True)
    scaler = torch.amp.GradScaler("cuda") if a.scaler else None
    B, S = a.batch_size, a.seq_len
    ids = torch.randint(0, 50257, (B, S), device=dev)
    inp, tg = ids[:, :-1], ids[:, 1:]
    pos = torch.arange(S - 1, device=dev).expand(B, -1)

    def step():
        opt.zero_grad(set_to_none=True)
        for _ in range(a.accum):
            with torch.autocast("cuda", dtype=torch.bfloat16):
                logits = call(inp, pos)
                loss = F.cross_entropy(logits.reshape(-1, 50257), tg.reshape(-1), ignore_index=-100) / a.accum
            if scaler is None:
                loss.backward()
            else:
                scaler.scale(loss).backward()
        if scaler is None:
            opt.step()
        else:
            scaler.step(opt)
            scaler.update()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    comm.barrier()
    dt = time.perf_counter() - t0
    tps = B * a.accum * (S - 1) * info.world_size * a.steps / dt
    if info.is_main:
        name = ("stock-pytorch" + ("-fsdp" if a.fsdp else "") + ("-sdpa" if a.sdpa else "-manual-attn")
                + ("-compile" if a.compile else ""))
        print(json.dumps({"baseline": name + ("-scaler" if a.scaler else ""),
                          "model": a.model, "n_gpus": info.world_size, "batch_per_gpu": B * a.accum,
                          "micro_batch": B, "accum": a.accum, "seq_len": S,
                          "tokens_per_s": round(tps, 1), "ms_per_step": round(1000 * dt / a.steps, 2),
                          "loss": round(loss.item(), 4),
                          "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 2)}))
    comm.cleanup_dist()


if __name__ == "__main__":
    main()
