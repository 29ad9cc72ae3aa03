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


# ---------------------------------------------------------------- peer-access collectives
def _ipc_input(p, n, dtype, salt=0):
    """Rank p's deterministic input of n elements (every rank can form every rank's)."""
    g = torch.Generator().manual_seed(1000 * p + 17 * n + salt)
    return torch.randn(n, generator=g).to(dtype).cuda()


def ipc_collectives_worker(rank, world, out):
    """Every collective of IpcComm on two ranks sharing cuda:0: exact against the rank-order f32
    sums, aligned and unaligned buffers, chunked (a small staging half) and not, f32 and bf16,
    and replayed from a HIP graph (the per-workgroup epochs advance on the device)."""
    _init()
    from distributed_pytorch_cookbook_amd.parallel.ipc_comm import IpcComm

    c = IpcComm(slot_mb=0.25, spin_limit=1 << 22)
    W = world

    def ref_sum(n, dtype, salt=0):
        acc = torch.zeros(n, device="cuda")
        for p in range(W):
            acc = acc + _ipc_input(p, n, dtype, salt).float()
        return acc.to(dtype)

    checked = 0
    for dtype in (torch.float32, torch.bfloat16):
        for n in (1, 63, 64, 1000, 4099, 300001):  # 300001 f32 > one 0.25 MiB half: chunked
            t = _ipc_input(rank, n, dtype)
            c.all_reduce(t)
            assert torch.equal(t, ref_sum(n, dtype)), ("all_reduce", dtype, n)
            # unaligned view (element-wise edges)
            big = torch.zeros(n + 1, dtype=dtype, device="cuda")
            big[1:] = _ipc_input(rank, n, dtype)
            c.all_reduce(big[1:])
            assert torch.equal(big[1:], ref_sum(n, dtype)), ("all_reduce unaligned", dtype, n)
            checked += 2
        for n in (1, 1000, 50000):
            full = [_ipc_input(p, W * n, dtype, 1) for p in range(W)]
            outp = torch.empty(n, dtype=dtype, device="cuda")
            c.reduce_scatter(outp, full[rank])
            exp = sum(f.float() for f in full).to(dtype)[rank * n:(rank + 1) * n]
            assert torch.equal(outp, exp), ("reduce_scatter", dtype, n)
            mine = _ipc_input(rank, n, dtype, 2)
            gath = torch.empty(W * n, dtype=dtype, device="cuda")
            c.all_gather(gath, mine)
            assert torch.equal(gath, torch.cat([_ipc_input(p, n, dtype, 2) for p in range(W)])), ("all_gather", dtype, n)
            b = _ipc_input(rank, n, dtype, 3)
            c.broadcast(b, src=1)
            assert torch.equal(b, _ipc_input(1, n, dtype, 3)), ("broadcast", dtype, n)
            checked += 3
    # copy-only collectives of any dtype (the pipeline's generation broadcasts int64 tokens)
    tok = torch.tensor([1000 + rank, -7, 1 << 40], dtype=torch.int64, device="cuda")
    c.broadcast(tok, src=1)
    assert tok.tolist() == [1001, -7, 1 << 40], ("broadcast int64", tok.tolist())
    g8 = torch.empty(W * 6, dtype=torch.uint8, device="cuda")
    c.all_gather(g8, torch.full((6,), 10 + rank, dtype=torch.uint8, device="cuda"))
    assert g8.tolist() == [10 + p for p in range(W) for _ in range(6)], ("all_gather uint8", g8.tolist())
    checked += 2
    # captured: two all-reduces per replay, new inputs each replay
    x = torch.empty(5000, device="cuda")
    y = torch.empty(777, dtype=torch.bfloat16, device="cuda")
    torch.cuda.synchronize()
    import torch.distributed as dist

    dist.barrier()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            c.all_reduce(x)
            c.all_reduce(y)
    for it in range(3):
        x.copy_(_ipc_input(rank, 5000, torch.float32, 10 + it))
        y.copy_(_ipc_input(rank, 777, torch.bfloat16, 20 + it))
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(x, ref_sum(5000, torch.float32, 10 + it)), ("graph f32", it)
        assert torch.equal(y, ref_sum(777, torch.bfloat16, 20 + it)), ("graph bf16", it)
        checked += 2
    # point-to-point: both directions in one group, two messages on one channel, a message larger
    # than a channel buffer (pieces), f32 and bf16, then three groups in a row on a channel
    cp = IpcComm(slot_mb=0.25, spin_limit=1 << 22, p2p_mb=0.0625)  # 64 KiB channels
    peer = rank ^ 1  # (pairs 0-1, 2-3, ...)
    for n, dtype in ((10, torch.float32), (100000, torch.float32), (77777, torch.bfloat16)):
        s1, s2 = _ipc_input(rank, n, dtype, 30), _ipc_input(rank, n // 2 + 1, dtype, 31)
        r1 = torch.empty(n, dtype=dtype, device="cuda")
        r2 = torch.empty(n // 2 + 1, dtype=dtype, device="cuda")
        cp.sendrecv(sends=[(s1, peer), (s2, peer)], recvs=[(r1, peer), (r2, peer)])
        torch.cuda.synchronize()
        assert torch.equal(r1, _ipc_input(peer, n, dtype, 30)) and torch.equal(r2, _ipc_input(peer, n // 2 + 1, dtype, 31)), ("p2p", n)
        checked += 2
    for it in range(3):  # one direction per group, alternating (the 1F1B pattern of two stages)
        t = _ipc_input(rank, 5000, torch.float32, 40 + it)
        r = torch.empty(5000, device="cuda")
        if (rank + it) % 2 == 0:
            cp.sendrecv(sends=[(t, peer)])
        else:
            cp.sendrecv(recvs=[(r, peer)])
            torch.cuda.synchronize()
            assert torch.equal(r, _ipc_input(peer, 5000, torch.float32, 40 + it)), ("p2p alternating", it)
            checked += 1
    # an empty message beside a non-empty one in one group (an empty tensor may have no pointer;
    # both sides still count it, so the channel stays in step)
    e_s, e_r = torch.empty(0, device="cuda"), torch.empty(0, device="cuda")
    t, r = _ipc_input(rank, 33, torch.float32, 45), torch.empty(33, device="cuda")
    cp.sendrecv(sends=[(e_s, peer), (t, peer)], recvs=[(e_r, peer), (r, peer)])
    torch.cuda.synchronize()
    assert torch.equal(r, _ipc_input(peer, 33, torch.float32, 45)), "p2p after an empty message"
    checked += 1
    # a stream of messages of different sizes on one channel (rank 1 -> 0): every half is reused with
    # a different split into workgroup sub-slices than its previous message (the FSDP checkpoint
    # gather's pattern), and the sender runs ahead of the receiver by up to two messages
    sizes = [200000, 1000, 150000, 70, 99999, 64, 180000, 3000, 120000, 5]
    if rank == 1:
        for k, n in enumerate(sizes):
            cp.sendrecv(sends=[(_ipc_input(1, n, torch.float32, 50 + k), 0)])
    elif rank == 0:
        for k, n in enumerate(sizes):
            r = torch.empty(n, device="cuda")
            cp.sendrecv(recvs=[(r, 1)])
            torch.cuda.synchronize()
            assert torch.equal(r, _ipc_input(1, n, torch.float32, 50 + k)), ("p2p stream", k, n)
            checked += 1
    torch.cuda.synchronize()
    cp.check()
    cp.destroy()
    c.check()
    c.destroy()
    if rank == 0:
        torch.save({"checked": checked}, out)


def ipc_engine_worker(rank, world, out, kind, steps, graph):
    """DDP / FSDP over the peer-access transport, two ranks on cuda:0, the step captured into a
    HIP graph on both ranks when ``graph``: the N > 1 capture path (collective capture decision,
    collectives recorded into the step graph, replays) run for real on one GPU."""
    info = _init()
    assert info.device.type == "cuda"
    from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine
    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine

    from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine

    m = make_model()
    if kind == "ddp":
        eng = DataParallelEngine(m, "cuda", lr=LR, bucket_mb=0.2, graph=graph, comm_kind="ipc")
        assert len(eng.store.buckets) >= 2
        tp, dp, rep = eng.store.tp, world, rank
    elif kind == "fsdp":
        eng = FSDPEngine(m, "cuda", lr=LR, prefetch=1, graph=graph, comm_kind="ipc")
        tp, dp, rep = eng.store.tp, world, rank
    else:  # pipeline over the peer-access point-to-point: "pipe-<schedule>"
        eng = PipelineEngine(m, "cuda", lr=LR, pp=world, dp=1, num_microbatches=4, schedule=kind.split("-")[1],
                             bucket_mb=0.2, seq_len=S - 1, graph=graph, comm_kind="ipc")
        tp, dp, rep = eng.pp_tp, 1, 0
    assert tp.kind == "ipc", tp.kind
    for s in range(steps):
        eng.train_step(*shard(*full_batch(step=s), rep, dp))
    torch.cuda.synchronize()
    if graph:
        assert eng._stepper.graph is not None, "the two-rank step was not captured"
    tp.nc.check()
    # the replicas / shards agree bit for bit across the ranks (each shard summed once, by its owner)
    sd = eng.full_state_dict()
    if rank == 0:
        torch.save({k: v.float().cpu() for k, v in sd.items()}, out)


def ipc_timeout_worker(rank, world, out):
    """A rank that never arrives: the peer's bounded waits give up, the kernel ends (no hung GPU),
    and check() names the failure."""
    _init()
    import torch.distributed as dist

    from distributed_pytorch_cookbook_amd.parallel.ipc_comm import IpcComm

    c = IpcComm(slot_mb=0.25, spin_limit=1 << 14)
    if rank == 0:
        t = torch.ones(1000, device="cuda")
        c.all_reduce(t)  # rank 1 never calls it
        torch.cuda.synchronize()
        try:
            c.check()
            raised = False
        except RuntimeError:
            raised = True
        torch.save({"raised": raised}, out)
    dist.barrier()
    c.destroy()
