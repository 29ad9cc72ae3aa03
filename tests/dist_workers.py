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


def worker_fsdp(rank, world, out, steps, prefetch, reshard, reduce_dtype="float32"):
    from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    m = make_model()
    eng = FSDPEngine(m, "cpu", lr=LR, prefetch=prefetch, reshard_after_forward=reshard,
                     reduce_dtype=getattr(torch, reduce_dtype))
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


def worker_pipe(rank, world, out, steps, pp, dp, micro, schedule, reduce_dtype="float32"):
    from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    m = make_model()
    eng = PipelineEngine(m, "cpu", lr=LR, pp=pp, dp=dp, num_microbatches=micro, schedule=schedule,
                         bucket_mb=0.01, seq_len=S, reduce_dtype=getattr(torch, reduce_dtype))
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


# ---------------------------------------------------------------- native communicator safety
def _use_fake(fake):
    import os

    os.environ["DPC_RCCL_LIB"] = fake
    os.environ["DPC_HIP_LIB"] = fake
    os.environ["DPC_WATCHDOG"] = "0"


def worker_native_fingerprint(rank, world, fake, log):
    """--coll_check on the NATIVE transport (the production path at N > 1): a rank enqueuing a
    differently shaped collective is caught before RCCL ever sees it."""
    import os

    _use_fake(fake)
    os.environ["FAKE_LOG"] = f"{log}.{rank}"
    from distributed_pytorch_cookbook_amd.parallel import comm
    from distributed_pytorch_cookbook_amd.parallel.transport import NativeTransport

    comm.init_dist(force_cpu=True)
    comm.set_coll_check(True)
    tp = NativeTransport(None, device="cpu")
    assert tp.kind == "native" and (tp.rank, tp.size) == (rank, world)
    tp.all_reduce(torch.ones(4))  # matched: reaches the (fake) RCCL
    tp.all_gather(torch.empty(8), torch.ones(4))
    try:
        tp.all_reduce(torch.ones(4 + rank))  # rank 1 differs
    except RuntimeError as exc:
        assert "collective mismatch" in str(exc), exc
        return
    raise AssertionError("mismatched native collective was not detected")


def worker_native_fingerprint_p2p(rank, world, fake, log):
    """--coll_check with pipeline p2p on the native transport: the ranks post DIFFERENT numbers
    of send/recv exchanges (as 1F1B does: M on the first stage, M + 1 on the last), then a
    matched all-reduce.  Point-to-point ops carry no group-wide fingerprint, so the later
    collective's fingerprints still pair up (no false mismatch, no hang)."""
    import os

    _use_fake(fake)
    os.environ["FAKE_LOG"] = f"{log}.{rank}"
    from distributed_pytorch_cookbook_amd.parallel import comm
    from distributed_pytorch_cookbook_amd.parallel.transport import NativeTransport

    comm.init_dist(force_cpu=True)
    comm.set_coll_check(True)
    tp = NativeTransport(None, device="cpu")
    peer = 1 - rank
    for _ in range(2 + rank):  # rank 0: 2 exchanges, rank 1: 3
        tp.sendrecv(sends=[(torch.ones(4), peer)], recvs=[(torch.empty(4), peer)])
    tp.all_reduce(torch.ones(4))
    tp.all_gather(torch.empty(8), torch.ones(4))


def worker_native_agreement(rank, world, fake, mode, log):
    """Native bring-up fails on ONE rank (rank 0 cannot draw the unique id, or rank 1's
    ncclCommInitRank fails): every rank refuses together -- nobody is left inside a native
    collective -- and the process group still works for the torch fallback."""
    import os

    import torch.distributed as dist

    _use_fake(fake)
    os.environ["FAKE_LOG"] = f"{log}.{rank}"
    if mode == "uid" and rank == 0:
        os.environ["FAKE_UID_FAIL"] = "1"
    if mode == "init" and rank == 1:
        os.environ["FAKE_INIT_FAIL"] = "1"
    from distributed_pytorch_cookbook_amd.parallel import comm
    from distributed_pytorch_cookbook_amd.parallel.native_comm import NativeComm

    comm.init_dist(force_cpu=True)
    try:
        NativeComm(None, device="cpu")
    except RuntimeError:
        pass
    else:
        raise AssertionError("expected every rank to refuse the native communicator")
    t = torch.ones(1)
    dist.all_reduce(t)
    assert t.item() == world


class _FailingCapture:
    """Stands in for ``torch.cuda.graph`` on CPU: the step body runs (as recording would)
    until the point where the gradient collectives have been launched, then the 'capture'
    fails, exactly as a capture error would surface on the GPU."""

    def __init__(self, eng):
        self.eng = eng
        self.saved = []

    def _boom(self, *a, **k):
        raise RuntimeError("simulated HIP-graph capture failure")

    def __enter__(self):
        st = self.eng.store
        tgt = st if hasattr(st, "finish_grads") and getattr(st, "tp", None) is not None else self.eng.p2p
        # FSDP's unit-wise path (finish_grads_and_update) and the bucket-by-bucket AdamW of DDP /
        # PP x DP (wait_bucket) fail at the same point
        names = ["finish_grads", "finish_grads_and_update", "wait_bucket"] if tgt is st else ["drain"]
        for name in names:
            if hasattr(tgt, name):
                self.saved.append((tgt, name))
                setattr(tgt, name, self._boom)
        return self

    def __exit__(self, *exc):
        for tgt, name in self.saved:
            delattr(tgt, name)  # back to the class method
        # on the GPU nothing a failed capture recorded ever runs; on CPU the collectives the
        # body issued did run: let them finish before the retry, or they would race with it
        st, p2p = self.eng.store, getattr(self.eng, "p2p", None)
        for h in list(getattr(st, "_works", {}).values()):
            h.wait()
        for lst in getattr(st, "_rs", {}).values():
            for h, _ in lst:
                h.wait()
        for _, w in getattr(st, "_full", {}).values():
            if w is not None:
                w.wait()
        for h in getattr(p2p, "_inflight", []):
            h.wait()
        return False


def worker_capture_fallback(rank, world, out, kind, inject, no_reset):
    """Three steps of an engine whose HIP-graph capture (step 2) fails part-way: the eager
    retry must give exactly the parameters of a never-graphed run."""
    from distributed_pytorch_cookbook_amd.engine.base import Engine
    from distributed_pytorch_cookbook_amd.parallel import comm

    comm.init_dist(force_cpu=True)
    if no_reset:  # negative control: the fallback without forgetting the failed step's state
        Engine.reset_step_state = lambda self: None
    m = make_model()
    if kind == "ddp":
        from distributed_pytorch_cookbook_amd.engine.data_parallel import DataParallelEngine

        eng = DataParallelEngine(m, "cpu", lr=LR, bucket_mb=0.02)
        dp, idx = world, rank
    elif kind == "fsdp":
        from distributed_pytorch_cookbook_amd.engine.fsdp import FSDPEngine

        eng = FSDPEngine(m, "cpu", lr=LR, prefetch=1)
        dp, idx = world, rank
    else:
        from distributed_pytorch_cookbook_amd.engine.pipeline import PipelineEngine

        pp = 2
        eng = PipelineEngine(m, "cpu", lr=LR, pp=pp, dp=world // pp, num_microbatches=2, bucket_mb=0.01, seq_len=S)
        dp, idx = world // pp, eng.replica
    if inject:
        eng.graph = True
        st = eng._stepper
        st._new_graph = lambda: object()
        st._capture = lambda g, mode: _FailingCapture(eng)
    for s in range(3):
        b, t = shard(*full_batch(step=s), idx, dp)
        eng.train_step(b, t)
    if inject:
        assert not eng._stepper.enabled  # it fell back to eager steps
    sd = eng.full_state_dict()
    if rank == 0:
        torch.save({k: v.clone() for k, v in sd.items()}, out)


def worker_fake_rccl_semantics(rank, world, fake, fake_dir):
    """NativeComm over the data-moving fake RCCL (tests/fakes/fake_rccl_hip.cpp, FAKE_DIR):
    every collective's result on every rank, grouped ring send/recv, and ncclCommSplit."""
    import os

    os.makedirs(fake_dir, exist_ok=True)
    _use_fake(fake)
    os.environ["FAKE_DIR"] = fake_dir
    from distributed_pytorch_cookbook_amd.parallel import comm
    from distributed_pytorch_cookbook_amd.parallel.native_comm import NativeComm

    comm.init_dist(force_cpu=True)
    c = NativeComm(None, device="cpu")
    assert (c.rank, c.size) == (rank, world)
    base = torch.arange(12, dtype=torch.float32) + 100 * rank
    # all-reduce sum / max / avg, f32, bf16 and int64
    t = base.clone()
    c.all_reduce(t)
    assert torch.equal(t, sum(torch.arange(12, dtype=torch.float32) + 100 * r for r in range(world)))
    t = base.clone()
    c.all_reduce(t, op="max")
    assert torch.equal(t, torch.arange(12, dtype=torch.float32) + 100 * (world - 1))
    t = base.clone()
    c.all_reduce(t, op="avg")
    assert torch.allclose(t, torch.arange(12, dtype=torch.float32) + 50 * (world - 1))
    tb = base.bfloat16()
    c.all_reduce(tb)
    assert torch.equal(tb, sum(torch.arange(12, dtype=torch.float32) + 100 * r for r in range(world)).bfloat16())
    ti = torch.full((3,), rank + 1, dtype=torch.int64)
    c.all_reduce(ti)
    assert ti.tolist() == [world * (world + 1) // 2] * 3
    # reduce-scatter: chunk `rank` of the summed input
    inp = torch.arange(4 * world, dtype=torch.float32) * (rank + 1)
    out = torch.empty(4)
    c.reduce_scatter(out, inp)
    scale = world * (world + 1) / 2
    assert torch.equal(out, torch.arange(4 * rank, 4 * rank + 4, dtype=torch.float32) * scale)
    # all-gather / broadcast
    g = torch.empty(3 * world)
    c.all_gather(g, torch.full((3,), float(rank)))
    assert g.tolist() == [float(r) for r in range(world) for _ in range(3)]
    bc = torch.full((5,), float(rank))
    c.broadcast(bc, src=2)
    assert bc.tolist() == [2.0] * 5
    # grouped ring exchange: send to the right, receive from the left (deadlock-free only
    # because the group posts every send first)
    right, left = (rank + 1) % world, (rank - 1) % world
    rx = torch.empty(6)
    for step in range(3):
        tx = torch.full((6,), float(10 * rank + step))  # (alive until the group has run)
        with c.grouped():
            c.send(tx, right)
            c.recv(rx, left)
        assert rx.tolist() == [float(10 * left + step)] * 6
    # 2 x 2 split: colour = rank // 2, key = -rank (reversed order inside a colour)
    sub = c.split(color=rank // 2, key=-rank)
    assert sub.size == 2 and sub.rank == 1 - rank % 2, (sub.rank, sub.size)
    s = torch.tensor([float(rank)])
    sub.all_reduce(s)
    lo = 2 * (rank // 2)
    assert s.item() == float(lo + lo + 1)
    # p2p on the split communicator: peer numbers are sub-communicator ranks
    peer = 1 - sub.rank
    got, tx = torch.empty(2), torch.tensor([float(rank), 7.0])
    with sub.grouped():
        sub.send(tx, peer)
        sub.recv(got, peer)
    assert got.tolist() == [float(lo + (1 - rank % 2)), 7.0]
    sub.destroy()
    c.destroy()


def worker_fake_rccl_p2p_completion(rank, world, fake, fake_dir):
    """RCCL's point-to-point completion rule in the fake (tests/fakes/fake_rccl_hip.cpp): a send
    completes only once the peer has received it.  Two ranks that each send, ungrouped, before
    they receive deadlock on xGMI; here that exchange must fail (time out) instead of passing,
    while the same exchange as one group (the pipeline engine's only form) completes."""
    import os

    os.makedirs(fake_dir, exist_ok=True)
    _use_fake(fake)
    os.environ["FAKE_DIR"] = fake_dir
    os.environ["FAKE_TIMEOUT_S"] = "4"
    from distributed_pytorch_cookbook_amd.parallel import comm
    from distributed_pytorch_cookbook_amd.parallel.native_comm import NativeComm

    comm.init_dist(force_cpu=True)
    c = NativeComm(None, device="cpu")
    peer = 1 - rank
    tx, rx = torch.full((4,), float(rank)), torch.empty(4)
    with c.grouped():  # the deadlock-free form
        c.send(tx, peer)
        c.recv(rx, peer)
    assert rx.tolist() == [float(peer)] * 4
    try:  # both ranks send first, ungrouped: each send waits for a receive that never comes
        c.send(tx, peer)
        c.recv(rx, peer)
    except RuntimeError as e:
        assert "failed" in str(e), e
    else:
        raise AssertionError("a mis-ordered ungrouped exchange completed: the fake does not model RCCL's blocking sends")
