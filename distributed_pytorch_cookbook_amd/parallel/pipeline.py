"""Pipeline parallelism: stage partitioning, GPipe / 1F1B schedules, p2p over RCCL.

Reference: ``/root/reference/main-pipe.py:21-83`` -- single-process
``torch.distributed.pipeline.sync.Pipe`` (removed from torch) with ``chunks =
num_stages`` micro-batches, stage i on ``cuda:i``, RPC initialised only because Pipe
needed it, and a layer split that is wrong as written (``:57-73``: the middle split is
overwritten in its loop, the last stage slices from the wrong index).  The intended
partition -- embeddings + first layers on stage 0, last layers + norm_out + lm_head on
the last stage, the rest spread over the middle -- is implemented correctly here and
*balanced by cost* (the lm_head of GPT-2 medium costs ~3.5 layers, so the last stage
gets fewer layers).

MI355X-first design: one process per GPU (torchrun), stage-to-stage activations
(the f32 residual stream [micro_batch * S, D], optionally bf16 on the wire) and their
gradients move with RCCL send/recv over the direct xGMI link between the two GPUs, issued
asynchronously on the transport's comm stream; paired send+recv are one grouped operation
(ncclGroupStart/End) so the 1F1B steady state cannot deadlock, and compute waits on a
receive only where it consumes it; the executed order is exactly ``schedule_1f1b`` /
``schedule_gpipe`` (``run_schedule``); the key-padding mask and targets are NOT sent --
every stage of a replica reads the same batch from its own loader.
"""
from __future__ import annotations

import torch


# Rates of the three kinds of work one training step does per token, measured on MI355X in
# the GPT-2 small DDP step (profiles/r4_final/ddp_kstats_final.md, pmc_ddp.md): GEMMs run
# ~1.0 PF/s (forward + input gradient + weight gradient = 3 x the forward FLOPs), flash
# attention ~0.4 PF/s (forward + backward = 3.5 x the forward FLOPs), the memory-bound
# kernels (LayerNorm fwd/bwd, residual / bias / activation passes, cross-entropy, embedding
# gather / scatter) ~5 TB/s.
_GEMM_RATE, _ATTN_RATE, _MEM_RATE = 1.0e15, 0.4e15, 5.0e12


def unit_costs(model, seq_len: int) -> list[float]:
    """Estimated seconds per token of one training step (forward + backward) for each unit
    (embeddings, layers..., head) -- the stage balance of ``partition``.  Counts the backward
    and the memory-bound passes, not only forward FLOPs: at GPT-2 small the head (LM-head GEMM
    + the cross-entropy over V logits) comes out at ~4.4 layers, at GPT-2 medium ~3.5."""
    D = model.dim
    hd = model.heads * model.head_dim
    V = model.vocab_size
    S = seq_len
    gemm = 2 * (3 * D * hd + hd * D + 2 * 4 * D * D)  # forward FLOPs of the layer's projections
    attn = 2 * S * hd  # causal: QK^T + PV over S / 2 keys on average
    layer_bytes = 32 * D + 4 * 4 * D  # two LayerNorms fwd + bwd, residual / bias / act' passes
    layer = 3 * gemm / _GEMM_RATE + 3.5 * attn / _ATTN_RATE + layer_bytes / _MEM_RATE
    # head: LM-head GEMM (3 x), the fused cross-entropy (read + write the bf16 logits), norm_out
    head = 3 * 2 * D * V / _GEMM_RATE + (4 * V + 16 * D) / _MEM_RATE
    emb = (4 * 4 * D + 64) / _MEM_RATE  # gather-add forward, sorted segment-sum backward
    return [emb] + [layer] * model.num_layers + [head]


def partition(costs: list[float], stages: int) -> list[list[int]]:
    """Contiguous split of units into ``stages`` groups minimising the max group cost
    (every group non-empty)."""
    n = len(costs)
    if stages > n:
        raise ValueError(f"cannot split {n} units into {stages} stages")
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)
    INF = float("inf")
    # best[k][i]: min max-cost splitting first i units into k groups
    best = [[INF] * (n + 1) for _ in range(stages + 1)]
    cut = [[0] * (n + 1) for _ in range(stages + 1)]
    best[0][0] = 0.0
    for k in range(1, stages + 1):
        for i in range(k, n + 1):
            for j in range(k - 1, i):
                v = max(best[k - 1][j], pre[i] - pre[j])
                if v < best[k][i]:
                    best[k][i], cut[k][i] = v, j
    groups = []
    i = n
    for k in range(stages, 0, -1):
        j = cut[k][i]
        groups.append(list(range(j, i)))
        i = j
    return groups[::-1]


class P2P:
    """Send/recv of fixed-shape activations between adjacent stages of one pipeline, through
    the pipeline's ``Transport`` (native RCCL on its comm stream by default).

    ``post`` enqueues ONE grouped exchange (ncclGroupStart/End) and returns immediately with
    the receive buffers and a handle: the compute stream waits on a receive only when it
    consumes it (``Recv.get``), and a send never blocks anything -- its buffer is kept alive
    by the transport until the comm stream has read it.  ``wire_dtype`` (e.g. bf16) halves
    the boundary bytes: activations / gradients are cast for the wire and back on arrival.
    """

    def __init__(self, tp, stage: int, n_stages: int, device, wire_dtype=None):
        self.tp = tp
        self.stage = stage
        self.n = n_stages
        self.device = device
        self.prev = stage - 1 if stage > 0 else None
        self.next = stage + 1 if stage < n_stages - 1 else None
        self.wire_dtype = wire_dtype
        self._inflight = []  # handles of exchanges nobody waits on yet (send-only groups)

    def post(self, send_next=None, send_prev=None, recv_prev_shape=None, recv_next_shape=None,
             dtype=torch.float32):
        """One grouped exchange.  Returns (Recv from prev or None, Recv from next or None)."""
        wdt = self.wire_dtype or dtype
        sends, recvs = [], []
        fp = fn = None
        if send_next is not None:
            sends.append((send_next.detach().to(wdt).contiguous(), self.next))
        if send_prev is not None:
            sends.append((send_prev.detach().to(wdt).contiguous(), self.prev))
        if recv_prev_shape is not None:
            fp = torch.empty(recv_prev_shape, device=self.device, dtype=wdt)
            recvs.append((fp, self.prev))
        if recv_next_shape is not None:
            fn = torch.empty(recv_next_shape, device=self.device, dtype=wdt)
            recvs.append((fn, self.next))
        h = self.tp.sendrecv(sends, recvs, async_op=True) if (sends or recvs) else None
        if h is not None and not recvs:
            self._inflight.append(h)  # a send is never waited on mid-step (see drain)
        return (Recv(fp, h, dtype) if fp is not None else None,
                Recv(fn, h, dtype) if fn is not None else None)

    def reset_step_state(self):
        """After a failed HIP-graph capture: the recorded sends never ran."""
        self._inflight.clear()

    def drain(self):
        """Order the caller after every send-only exchange still in flight (end of a step:
        device-side for RCCL; for gloo it also keeps the works alive until they complete)."""
        for h in self._inflight:
            h.wait()
        self._inflight.clear()

    def exchange(self, send_next=None, send_prev=None, recv_prev_shape=None, recv_next_shape=None,
                 dtype=torch.float32):
        """Blocking form of ``post`` (waits for the received tensors and the sends)."""
        a, b = self.post(send_next, send_prev, recv_prev_shape, recv_next_shape, dtype)
        out = (a.get() if a is not None else None), (b.get() if b is not None else None)
        self.drain()
        return out


class Recv:
    """A receive buffer whose data is ready once its exchange's handle has been waited on."""

    def __init__(self, buf, handle, dtype):
        self.buf, self.handle, self.dtype = buf, handle, dtype

    def get(self):
        if self.handle is not None:
            self.handle.wait()
            self.handle = None
        return self.buf if self.buf.dtype == self.dtype else self.buf.to(self.dtype)


def run_schedule(order, first: bool, last: bool, forward, backward, p2p: "P2P", shape):
    """Execute a stage's schedule -- a list of ('F', m) / ('B', m) from ``schedule_1f1b`` or
    ``schedule_gpipe`` -- with asynchronous grouped p2p.

    Rule: before the first op its receive is posted; after every op ONE grouped exchange is
    posted holding that op's send (y_m to the next stage, dx_m to the previous) and the
    receive the NEXT op will consume (x from the previous stage for an F, g from the next
    for a B).  Every exchange is issued in schedule order on both sides of a link, so the
    comm streams see the same group sequence the blocking PipeDream-flush loop issues --
    deadlock-free -- while the compute stream waits only where a received tensor is used.
    ``forward(m, x) -> y`` (None on the last stage), ``backward(m, g) -> dx`` (None on the
    first stage)."""

    def need(op):
        kind, _ = op
        if kind == "F":
            return (shape, None) if not first else (None, None)
        return (None, shape) if not last else (None, None)

    pending = None  # the Recv the next op consumes
    rp, rn = need(order[0]) if order else (None, None)
    if rp is not None or rn is not None:
        a, b = p2p.post(recv_prev_shape=rp, recv_next_shape=rn)
        pending = a or b
    for i, (kind, m) in enumerate(order):
        if kind == "F":
            x = pending.get() if (pending is not None and not first) else None
            out = forward(m, x)
            send_next, send_prev = (out if not last else None), None
        else:
            g = pending.get() if (pending is not None and not last) else None
            dx = backward(m, g)
            send_next, send_prev = None, (dx if not first else None)
        pending = None
        rp = rn = None
        if i + 1 < len(order):
            rp, rn = need(order[i + 1])
        if send_next is not None or send_prev is not None or rp is not None or rn is not None:
            a, b = p2p.post(send_next=send_next, send_prev=send_prev, recv_prev_shape=rp,
                            recv_next_shape=rn)
            pending = a or b
    p2p.drain()


def schedule_1f1b(n_micro: int, stage: int, n_stages: int):
    """List of ('F', m) / ('B', m) in execution order for one stage (PipeDream-flush)."""
    warm = min(n_stages - stage - 1, n_micro)
    order = [("F", m) for m in range(warm)]
    f, b = warm, 0
    while f < n_micro:
        order.append(("F", f))
        f += 1
        order.append(("B", b))
        b += 1
    while b < n_micro:
        order.append(("B", b))
        b += 1
    return order


def schedule_gpipe(n_micro: int, stage: int, n_stages: int):
    return [("F", m) for m in range(n_micro)] + [("B", m) for m in range(n_micro)]
