"""Worker bodies for the multi-process engine tests (importable by spawned children)."""
from __future__ import annotations

import torch

V, S, D, H, HD, L = 97, 24, 32, 2, 16, 3
LR = 1e-2


def make_model(seed=0, act="relu", layers=L):
    from distributed_pytorch_cookbook_amd.models.gpt import TransformerDecoderLM

    torch.manual_seed(seed)
    return TransformerDecoderLM(dim=D, head_dim=HD, heads=H, num_layers=layers, vocab_size=V,
                                max_position_embeddings=S, activation=act)


def full_batch(N=8, seed=3, step=0):
    g = torch.Generator().manual_seed(seed + 17 * step)
    ids = torch.randint(0, V, (N, S), generator=g)
    inputs, targets = ids[:, :-1].contiguous(), ids[:, 1:].contiguous()
    pos = torch.arange(S - 1).unsqueeze(0).expand(N, -1).contiguous()
    return dict(input_ids=inputs, position_ids=pos, mask=None), targets


def shard(batch, targets, i, n):
    N = targets.shape[0]
    sl = slice(i * N // n, (i + 1) * N // n)
    return {k: (v[sl] if torch.is_tensor(v) else v) for k, v in batch.items()}, targets[sl]


def reference_state(steps=2, layers=L):
    """Single-process result on the full batch."""
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine

    m = make_model(layers=layers)
    eng = DataParallelEngine(m, "cpu", lr=LR)
    losses = []
    for s in range(steps):
        b, t = full_batch(step=s)
        losses.append(float(eng.train_step(b, t)))
    return {k: v.clone() for k, v in eng.full_state_dict().items()}, losses


def worker_ddp(rank, world, out, steps, bucket_mb, reduce_dtype):
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    m = make_model()
    eng = DataParallelEngine(m, "cpu", lr=LR, bucket_mb=bucket_mb,
                             reduce_dtype=getattr(torch, reduce_dtype))
    assert len(eng.store.buckets) >= 2 or bucket_mb > 1
    for s in range(steps):
        b, t = shard(*full_batch(step=s), rank, world)
        eng.train_step(b, t)
    sd = eng.full_state_dict()
    if rank == 0:
        torch.save({k: v.clone() for k, v in sd.items()}, out)


def worker_fsdp(rank, world, out, steps, prefetch, reshard):
    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    m = make_model()
    eng = FSDPEngine(m, "cpu", lr=LR, prefetch=prefetch, reshard_after_forward=reshard)
    for s in range(steps):
        b, t = shard(*full_batch(step=s), rank, world)
        eng.train_step(b, t)
    sd = eng.full_state_dict()
    # eval + generation must run collectively without hanging
    with torch.no_grad():
        b, t = shard(*full_batch(step=99), rank, world)
        r = eng.eval_step(b, t)
        assert r[1].item() > 0
    if rank == 0:
        torch.save(sd, out)


def worker_pipe(rank, world, out, steps, pp, dp, micro, schedule):
    from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    m = make_model()
    eng = PipelineEngine(m, "cpu", lr=LR, pp=pp, dp=dp, num_microbatches=micro, schedule=schedule,
                         bucket_mb=0.01, seq_len=S)
    losses = []
    for s in range(steps):
        b, t = shard(*full_batch(step=s), eng.replica, dp)
        loss = eng.train_step(b, t)
        losses.append(None if loss is None else float(loss))
    sd = eng.full_state_dict()
    # eval and a generate-style forward must stay matched on every rank
    b, t = shard(*full_batch(step=99), eng.replica, dp)
    eng.eval_step(b, t)
    f = eng.lm()
    ids = torch.randint(0, V, (1, 5))
    f(input_ids=ids, position_ids=torch.arange(5).unsqueeze(0))
    if rank == 0:
        torch.save({"sd": sd, "groups": eng.groups}, out)


def worker_scaled(rank, world, out, kind):
    """--grad_scaler on each engine kind (DDP / FSDP / pipeline): a 2^16-scaled backward with
    the unscale folded into AdamW must land on the unscaled result."""
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine
    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine
    from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    m = make_model()
    if kind == "ddp":
        eng = DataParallelEngine(m, "cpu", lr=LR, bucket_mb=0.05, grad_scaler=True)
    elif kind == "fsdp":
        eng = FSDPEngine(m, "cpu", lr=LR, grad_scaler=True)
    else:
        eng = PipelineEngine(m, "cpu", lr=LR, pp=world, dp=1, num_microbatches=2, bucket_mb=0.01, seq_len=S,
                             grad_scaler=True)
    dp, idx = (1, 0) if kind == "pipe" else (world, rank)
    for s in range(2):
        b, t = shard(*full_batch(step=s), idx, dp)
        eng.train_step(b, t)
    assert float(eng.scaler.tracker) == 2.0
    sd = eng.full_state_dict()
    if rank == 0:
        torch.save({k: v.clone() for k, v in sd.items()}, out)


def worker_coll_mismatch(rank, world):
    """DPC_COLL_CHECK: a rank issuing a differently shaped collective is caught by the
    fingerprint exchange (on every rank) instead of hanging or corrupting the reduction."""
    import os

    os.environ["DPC_COLL_CHECK"] = "1"
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    comm.all_reduce(torch.ones(4))  # matched: passes
    try:
        comm.all_reduce(torch.ones(4 + rank))  # rank 1 differs
    except RuntimeError as exc:
        assert "collective mismatch" in str(exc), exc
        return
    raise AssertionError("mismatched collective was not detected")


def worker_fsdp_mem(rank, world, out):
    """Peak number of full-unit buffers alive in the FSDP store over one training step."""
    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    res = {}
    for prefetch in (0, 1, 2):
        m = make_model(layers=5)
        eng = FSDPEngine(m, "cpu", lr=LR, prefetch=prefetch)
        b, t = shard(*full_batch(step=0), rank, world)
        eng.train_step(b, t)
        res[prefetch] = eng.store.peak_live_units
    if rank == 0:
        torch.save(res, out)


def worker_stream_check(rank, world, out, kind):
    """--stream_check: every engine's step leaves no collective un-waited, and
    an async collective nobody waits on is reported at the end of the step."""
    from distributed_pytorch_cookbook_amd.parallel import comm, transport

    comm.init_dist(force_cpu=True)
    transport.set_stream_check(True)
    m = make_model()
    if kind == "ddp":
        from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine

        eng = DataParallelEngine(m, "cpu", lr=LR, bucket_mb=0.05)
    elif kind == "fsdp":
        from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine

        eng = FSDPEngine(m, "cpu", lr=LR, prefetch=1)
    else:
        from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine

        eng = PipelineEngine(m, "cpu", lr=LR, pp=world, dp=1, num_microbatches=4, schedule="1f1b",
                             bucket_mb=0.01, seq_len=S)
    for s in range(2):
        b, t = full_batch(step=s) if kind == "pipe" else shard(*full_batch(step=s), rank, world)
        eng.train_step(b, t)  # raises if the engine left a collective un-waited
    tp = transport.TorchTransport()
    x = torch.ones(4)
    h = tp.all_reduce(x, async_op=True)
    caught = False
    try:
        transport.check_drained("the test's end")
    except RuntimeError as exc:
        caught = "all_reduce(4,)" in str(exc)
    h.wait()  # (the collective itself still completes on every rank)
    transport.check_drained("after the wait")  # nothing outstanding now
    if rank == 0:
        torch.save({"caught": caught}, out)
