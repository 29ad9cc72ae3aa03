"""Worker bodies for the multi-rank GPU engine tests: every rank runs the real HIP kernels on
cuda:0 and the ranks talk over gloo (``DPC_DIST_BACKEND=gloo``) -- RCCL refuses two ranks
on one GPU, and a test box has one.  Importable by spawned children."""
from __future__ import annotations

import os

import torch

V, S, D, H, HD, L = 1000, 64, 128, 2, 64, 3
LR = 1e-3


def make_model(seed=0):
    from distributed_pytorch_cookbook_amd.models.gpt import TransformerDecoderLM

    torch.manual_seed(seed)
    with torch.device("cuda"):
        return TransformerDecoderLM(dim=D, head_dim=HD, heads=H, num_layers=L, vocab_size=V,
                                    max_position_embeddings=S, activation="gelu")


def full_batch(N=8, step=0):
    g = torch.Generator().manual_seed(7 + 13 * step)
    ids = torch.randint(0, V, (N, S), generator=g).cuda()
    pos = torch.arange(S - 1, device="cuda").unsqueeze(0).expand(N, -1)
    return dict(input_ids=ids[:, :-1], position_ids=pos, mask=None), ids[:, 1:]


def shard(batch, targets, i, n):
    N = targets.shape[0]
    sl = slice(i * N // n, (i + 1) * N // n)
    return {k: (v[sl] if torch.is_tensor(v) else v) for k, v in batch.items()}, targets[sl]


def reference_state(steps=3):
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine

    eng = DataParallelEngine(make_model(), "cuda", lr=LR)
    losses = [float(eng.train_step(*full_batch(step=s))) for s in range(steps)]
    return {k: v.float().cpu() for k, v in eng.full_state_dict().items()}, losses


def _init():
    os.environ["DPC_DIST_BACKEND"] = "gloo"
    from distributed_pytorch_cookbook_amd.parallel import comm

    return comm.init_dist()


def worker(rank, world, out, kind, steps, opts):
    info = _init()
    assert info.device.type == "cuda"
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine
    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine
    from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine

    m = make_model()
    if kind == "ddp":
        eng = DataParallelEngine(m, "cuda", lr=LR, bucket_mb=opts.get("bucket_mb", 0.2),
                                 reduce_dtype=getattr(torch, opts.get("reduce_dtype", "float32")))
        assert len(eng.store.buckets) >= 2
        dp, rep = world, rank
    elif kind == "fsdp":
        eng = FSDPEngine(m, "cuda", lr=LR, prefetch=opts.get("prefetch", 1))
        dp, rep = world, rank
    else:
        eng = PipelineEngine(m, "cuda", lr=LR, pp=opts["pp"], dp=opts["dp"], num_microbatches=opts["micro"],
                             schedule=opts.get("schedule", "1f1b"), bucket_mb=0.2, seq_len=S - 1)
        dp, rep = opts["dp"], eng.replica
    for s in range(steps):
        eng.train_step(*shard(*full_batch(step=s), rep, dp))
    torch.cuda.synchronize()
    sd = eng.full_state_dict()  # gathered to rank 0 (None elsewhere for FSDP / pipeline)
    if rank == 0:
        torch.save({k: v.float().cpu() for k, v in sd.items()}, out)
