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
``schedule_gpipe`` / ``schedule_zb`` (``run_schedule``); the key-padding mask and targets are
NOT sent -- every stage of a replica reads the same batch from its own loader.

Zero-bubble schedule (``schedule_zb``, Qi et al. 2023 "Zero Bubble Pipeline Parallelism",
the H1 family): a micro-batch's backward is split into B -- the input-gradient chain, what the
previous stage waits for -- and W -- the weight-gradient GEMMs (and the embedding scatter),
which nothing downstream needs.  W passes are deferred into the slots where 1F1B idles (an
early stage waiting for gradients to come back), so the cooldown bubble is filled with work
the step has to do anyway.  The per-stage orders come from an event simulation of every stage
under a per-stage cost model (``simulate_orders``), identical on all ranks; the F / B
relative order is 1F1B's.  HBM is plentiful on MI355X (288 GB), so a stage may hold up to
``wmax`` deferred W passes (their dY / X operands) beside 1F1B's in-flight activations.
"""
from __future__ import annotations

import functools
import heapq

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


def run_schedule(order, first: bool, last: bool, forward, backward, p2p: "P2P", shape, wgrad=None):
    """Execute a stage's schedule -- a list of ('F', m) / ('B', m) from ``schedule_1f1b`` or
    ``schedule_gpipe``, plus ('W', m) from ``schedule_zb`` (``wgrad(m)``: the deferred weight
    gradients of micro-batch m; no communication) -- with asynchronous grouped p2p.

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
        if kind == "W":
            return (None, None)
        return (None, shape) if not last else (None, None)

    pending = None  # the Recv the next op consumes
    rp, rn = need(order[0]) if order else (None, None)
    if rp is not None or rn is not None:
        a, b = p2p.post(recv_prev_shape=rp, recv_next_shape=rn)
        pending = a or b
    for i, (kind, m) in enumerate(order):
        if kind == "W":
            wgrad(m)
            send_next = send_prev = None
        elif kind == "F":
            x = pending.get() if (pending is not None and not first) else None
            out = forward(m, x)
            send_next, send_prev = (out if not last else None), None
        else:
            g = pending.get() if (pending is not None and not last) else None
            dx = backward(m, g)
            send_next, send_prev = None, (dx if not first else None)
        if kind != "W":  # (a W consumes nothing: a receive posted before it stays pending)
            pending = None
        rp = rn = None
        # the receive of the next op that communicates goes into THIS op's group, W passes in
        # between or not: a send-only group followed by a receive-only group on both sides of a
        # link deadlocks under RCCL's blocking sends (p2p_deadlock_free)
        j = i + 1
        while j < len(order) and order[j][0] == "W":
            j += 1
        if j < len(order) and pending is None:
            rp, rn = need(order[j])
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


# ---------------------------------------------------------------- zero-bubble (B / W split)
def stage_costs(model, seq_len: int, groups) -> list[tuple[float, float, float]]:
    """(F, B, W) seconds per token of each stage's units under the ``unit_costs`` rates: B is the
    input-gradient chain (dgrad GEMMs, the attention backward ~2.5 x its forward, the memory
    passes), W the weight-gradient GEMMs (the LM head's included: the largest single product of
    the last stage) and the embedding scatter."""
    D = model.dim
    hd = model.heads * model.head_dim
    V = model.vocab_size
    S = seq_len
    g = 2 * (3 * D * hd + hd * D + 2 * 4 * D * D) / _GEMM_RATE
    a = 2 * S * hd / _ATTN_RATE
    mem = (32 * D + 4 * 4 * D) / _MEM_RATE
    per_unit = {}
    L = model.num_layers
    for u in range(L + 2):
        if u == 0:
            per_unit[u] = (4 * D / _MEM_RATE, 0.0, (8 * D + 64) / _MEM_RATE)
        elif u == L + 1:
            hg = 2 * D * V / _GEMM_RATE
            per_unit[u] = (hg + 2 * V / _MEM_RATE, hg + (2 * V + 16 * D) / _MEM_RATE, hg)
        else:
            per_unit[u] = (g + a + 0.4 * mem, g + 2.5 * a + 0.6 * mem, g)
    return [tuple(sum(per_unit[u][k] for u in grp) for k in range(3)) for grp in groups]


def fb_order(n_micro: int, stage: int, n_stages: int, warm: int | None = None):
    """1F1B's F / B order for one stage with ``warm`` forwards before the first backward (default
    stages - stage - 1, PipeDream-flush)."""
    w = n_stages - stage - 1 if warm is None else warm
    return [op for op in schedule_1f1b_w(n_micro, min(max(w, 0), n_micro))]


def schedule_1f1b_w(n_micro: int, warm: int):
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


def simulate_orders(n_micro: int, costs, wmax=None, comm: float = 0.0, split_w: bool = True, warm=None):
    """Event simulation of a pipeline step: per-stage op orders and finish times.

    ``costs[s] = (F, B, W)`` per micro-batch on stage s.  Every stage runs 1F1B's F / B order
    (``warm[s]`` forwards before its first backward, default stages - s - 1) -- the order whose
    grouped p2p is deadlock-free under RCCL's blocking sends (``p2p_deadlock_free``; W passes do
    not communicate, so where they sit cannot change that) -- and places the W passes: whenever
    its next F / B has not received its input yet, a stage runs its oldest deferred W; it also
    runs one first when it already holds more than ``wmax[s]`` (default stages) deferred W
    passes (their dY / X operands stay resident); the rest run after its last B.
    ``split_w=False`` runs each W right after its B (= 1F1B with B + W as one backward).
    Returns (orders, makespan, busy per stage).  Deterministic: every rank derives the same
    orders."""
    p = len(costs)
    if wmax is None:
        wmax = [p] * p
    fbs = [fb_order(n_micro, s, p, None if warm is None else warm[s]) for s in range(p)]
    INF = float("inf")
    t = [0.0] * p
    nxt = [0] * p  # index of the stage's next F / B op
    wq = [[] for _ in range(p)]
    fin = {}  # (kind, stage, m) -> finish time
    orders = [[] for _ in range(p)]
    busy = [0.0] * p

    def ready_at(s):
        """Arrival time of the input of stage s's next F / B (INF: not scheduled yet)."""
        if nxt[s] >= len(fbs[s]):
            return INF
        kind, m = fbs[s][nxt[s]]
        if kind == "F":
            return 0.0 if s == 0 else fin.get(("F", s - 1, m), INF) + comm
        if s == p - 1:
            return fin.get(("F", s, m), INF)
        return fin.get(("B", s + 1, m), INF) + comm

    def run(s, kind, m, c):
        orders[s].append((kind, m))
        t[s] += c
        busy[s] += c
        fin[(kind, s, m)] = t[s]

    while True:
        best = None
        for s in range(p):
            if nxt[s] >= len(fbs[s]) and not wq[s]:
                continue
            start = t[s] if wq[s] else max(t[s], ready_at(s))
            if start < INF and (best is None or start < best[0]):
                best = (start, s)
        if best is None:
            if any(nxt[s] < len(fbs[s]) or wq[s] for s in range(p)):
                raise RuntimeError("pipeline simulation stalled")
            break
        start, s = best
        t[s] = start
        F, B, W = costs[s]
        if wq[s] and (len(wq[s]) > wmax[s] or ready_at(s) > t[s]):
            run(s, "W", wq[s].pop(0), W)
            continue
        kind, m = fbs[s][nxt[s]]
        nxt[s] += 1
        run(s, kind, m, F if kind == "F" else B)
        if kind == "B":
            if split_w:
                wq[s].append(m)
            else:
                run(s, "W", m, W)
    return orders, max(t), busy


def zb_limits(n_micro: int, n_stages: int, mem: int = 1):
    """(wmax, warm) per stage of the zero-bubble policies: mem 1 = H1 (1F1B's warm-up, at most
    ``stages`` deferred W passes); mem 2 = H2-like (twice 1F1B's forwards in flight -- warm-up
    2 (stages - s) - 1, still deadlock-free, p2p_deadlock_free; 3x is not -- and every W deferrable:
    the early stages run most of their W passes after their last B, so the later stages'
    start-up bubble is not repeated at the end; more HBM, which MI355X has)."""
    p = n_stages
    if mem == 1:
        return [p] * p, [p - s - 1 for s in range(p)]
    return [n_micro] * p, [2 * (p - s) - 1 for s in range(p)]


@functools.lru_cache(maxsize=64)
def _zb_orders(n_micro: int, costs: tuple, wmax: tuple | None, mem: int = 1):
    wm, warm = zb_limits(n_micro, len(costs), mem)
    orders, _, _ = simulate_orders(n_micro, list(costs), list(wmax) if wmax else wm, warm=warm)
    return tuple(tuple(o) for o in orders)


def schedule_zb(n_micro: int, stage: int, n_stages: int, costs=None, wmax=None, mem: int = 1):
    """('F', m) / ('B', m) / ('W', m) in execution order for one stage: the zero-bubble schedule
    of ``simulate_orders`` (``costs``: per-stage (F, B, W), default equal thirds; ``mem``: the
    memory policy of ``zb_limits``)."""
    c = tuple(tuple(x) for x in costs) if costs is not None else ((1.0, 1.0, 1.0),) * n_stages
    if len(c) != n_stages:
        raise ValueError("schedule_zb: one (F, B, W) cost triple per stage")
    return list(_zb_orders(n_micro, c, tuple(wmax) if wmax is not None else None, mem)[stage])


def bubble_factor(n_micro: int, costs, schedule: str = "zb", comm: float = 0.0) -> float:
    """Modelled step time over the busiest stage's work (1.0 = no bubble) for 1F1B (B + W as one
    backward) or the zero-bubble orders ("zb" / "zb2"), under the cost model -- the proxy's
    bubble term."""
    if schedule == "1f1b":
        _, span, busy = simulate_orders(n_micro, costs, comm=comm, split_w=False)
    else:
        wm, warm = zb_limits(n_micro, len(costs), 2 if schedule == "zb2" else 1)
        _, span, busy = simulate_orders(n_micro, costs, wmax=wm, comm=comm, warm=warm)
    return span / max(busy)


def p2p_deadlock_free(orders) -> bool:
    """Check a set of per-stage orders against RCCL's point-to-point semantics as
    ``run_schedule`` issues them: after op i one group holding op i's send and the receive the
    next communicating op consumes (the first op's receive alone before it); a group completes only when every
    send in it has been matched by the peer's receive in the peer's CURRENT group and every
    receive by the peer's send.  True when every stage runs to the end."""
    p = len(orders)
    groups = []
    for s, order in enumerate(orders):
        first, last = s == 0, s == p - 1

        def need(op):
            if op[0] == "F":
                return None if first else ("recv", s - 1, ("F", op[1]))
            if op[0] == "B":
                return None if last else ("recv", s + 1, ("B", op[1]))
            return None

        gs = []
        pend = need(order[0]) if order else None  # (a schedule never starts with a W)
        if pend:
            gs.append([pend])
        for i, op in enumerate(order):
            g = []
            if op[0] == "F" and not last:
                g.append(("send", s + 1, ("F", op[1])))
            if op[0] == "B" and not first:
                g.append(("send", s - 1, ("B", op[1])))
            if op[0] != "W":
                pend = None
            j = i + 1
            while j < len(order) and order[j][0] == "W":
                j += 1
            if j < len(order) and pend is None:
                pend = need(order[j])
                if pend:
                    g.append(pend)
            if g:
                gs.append(g)
        groups.append(gs)
    cur = [0] * p
    left = [set(range(len(groups[s][0]))) if groups[s] else set() for s in range(p)]
    progress = True
    while progress:
        progress = False
        for s in range(p):
            if cur[s] >= len(groups[s]):
                continue
            g = groups[s][cur[s]]
            for j in list(left[s]):
                kind, peer, msg = g[j]
                if cur[peer] >= len(groups[peer]):
                    continue
                pg = groups[peer][cur[peer]]
                want = ("recv" if kind == "send" else "send", s, msg)
                for k in list(left[peer]):
                    if pg[k] == want:
                        left[s].discard(j)
                        left[peer].discard(k)
                        progress = True
                        break
            for q in (s,) + tuple(x for x in (s - 1, s + 1) if 0 <= x < p):
                while cur[q] < len(groups[q]) and not left[q]:
                    cur[q] += 1
                    if cur[q] < len(groups[q]):
                        left[q] = set(range(len(groups[q][cur[q]])))
                    progress = True
    return all(cur[s] >= len(groups[s]) for s in range(p))
