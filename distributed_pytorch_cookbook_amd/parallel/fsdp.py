"""Fully-sharded data parallel (ZeRO-3) store: per-unit flat shards over RCCL.

Reference: ``FSDP(sp_model, auto_wrap_policy=size_based(min_num_params=100),
cpu_offload=CPUOffload(offload_params=...))`` (``/root/reference/main-fsdp.py:60-69``),
which makes every leaf Linear / Embedding / LayerNorm its own unit (8L+5 units: 389 for
GPT-2 XL) and all-gathers fp32 parameters.

MI355X-first design:
* one unit per decoder layer (+ embeddings, + head): GPT-2 XL has 50 units of up to
  30.7M parameters -- few, large collectives that run at RCCL's bus bandwidth over xGMI
  instead of hundreds of latency-bound ones;
* every rank owns a contiguous 1/W slice of each unit (padded to W x 64 elements) in
  f32 (master) + f32 (gradient) + bf16 (compute copy written by the AdamW kernel);
* forward / backward all-gather the *bf16* shards (half the bytes of the reference's
  fp32 gathers) into a full-unit buffer, prefetched ``prefetch`` units ahead on RCCL's
  stream while the current unit computes; buffers are released after use
  (``reshard_after_forward``) so activation-time memory holds only the prefetch window;
* backward reduce-scatters each unit's f32 gradient straight into the shard gradient
  as soon as the unit's backward has written it (overlapped with the next unit), and the
  full-unit gradient is dropped the moment its reduce-scatter is enqueued (the transport
  ``record_stream``s it, so the allocator recycles it once the collective has read it):
  gradient memory is the shards plus the units in flight, not the whole model;
* with one rank the unit buffers ARE the shards (no gathers, no copies) and the weight
  gradients accumulate straight into the shard gradient;
* collectives ride the engine's ``Transport`` (native RCCL on a side stream by default);
* ``cpu_offload``: master shard and Adam moments live in pinned host memory, the
  optimizer runs on the host, the bf16 shard is copied back asynchronously.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops.elementwise import cast_f32_bf16
from . import comm
from .store import ALIGN, FlatLayout, ParamStore, default_compute_dtype
from .transport import Transport, make_transport
from ..utils.profiling import mark


def _placeholder(shape, device):
    """A tensor with the parameter's shape but one element of storage (the real data
    lives in the shards)."""
    return torch.empty(1, device=device).expand(*shape) if len(shape) else torch.empty((), device=device)


class FSDPStore(ParamStore):
    def __init__(self, model, device, group=None, compute_dtype=None, prefetch: int = 1,
                 reshard_after_forward: bool = True, cpu_offload: bool = False,
                 reduce_dtype: torch.dtype = torch.float32, transport: Transport | None = None,
                 comm_kind: str | None = None, force_sharded: bool = False):
        self.device = torch.device(device)
        self.group = group
        self.tp = transport if transport is not None else make_transport(group, self.device, comm_kind)
        self.W = self.tp.size
        # the N > 1 code path (full-unit gathers, unit gradients, reduce-scatters) even at one
        # rank: bench.py --force_dist_path profiles it on a single GPU
        self.sharded = self.W > 1 or force_sharded
        self.rank = self.tp.rank
        self.compute_dtype = compute_dtype or default_compute_dtype(self.device)
        self.prefetch = max(0, prefetch)
        self.reshard = reshard_after_forward
        self.cpu_offload = cpu_offload and self.device.type == "cuda"
        self.reduce_dtype = reduce_dtype
        self.layout = FlatLayout(model, unit_align=self.W * ALIGN)
        self.nunits = len(self.layout.units)
        self.units = list(range(self.nunits))
        # shard geometry
        self.unit_len = [b - a for a, b in self.layout.unit_ranges]
        self.shard_len = [n // self.W for n in self.unit_len]
        self.shard_off = [0]
        for n in self.shard_len[:-1]:
            self.shard_off.append(self.shard_off[-1] + n)
        total = sum(self.shard_len)
        host = self.cpu_offload
        self._host_tasks = {}  # --cpu_offload: unit -> Future of the event after its shadow upload
        self._d2h_done = None  # event after the step's gradient copies (zero_grad waits on it)
        mdev = torch.device("cpu") if host else self.device
        self.master = torch.zeros(total, dtype=torch.float32, device=mdev,
                                  pin_memory=host)
        self.grads = torch.zeros(total, dtype=torch.float32, device=self.device)
        self.grads_host = torch.zeros(total, dtype=torch.float32, pin_memory=True) if host else None
        self.shadow = torch.empty(total, dtype=self.compute_dtype, device=self.device)
        # 1-D parameters (biases, LayerNorm affine: ~0.1% of the model) stay REPLICATED in f32
        # like DDP parameters: the kernels read them in f32 (a bf16-gathered LayerNorm gain
        # near 1.0 would round away every update smaller than 2^-8) and their gradients are
        # all-reduced once per step in a single small collective.
        self.rep = [e for e in self.layout.entries if len(e.shape) < 2]
        self.rep_off = {}
        off = 0
        for e in self.rep:
            self.rep_off[id(e.param)] = off
            off += (e.numel + 63) // 64 * 64
        self.rep_master = torch.zeros(max(off, 64), dtype=torch.float32, device=self.device)
        self.rep_grads = torch.zeros_like(self.rep_master)
        with torch.no_grad():
            for e in self.rep:
                o = self.rep_off[id(e.param)]
                self.rep_master[o:o + e.numel].copy_(e.param.data.reshape(-1))
        # fill my shards from the (identically seeded) full parameters, then free them
        with torch.no_grad():
            for u in self.units:
                lo, hi = self.layout.unit_ranges[u]
                mine0 = lo + self.rank * self.shard_len[u]
                mine1 = mine0 + self.shard_len[u]
                for e in self.layout.unit_entries(u):
                    a, b = max(e.offset, mine0), min(e.offset + e.numel, mine1)
                    if a < b:
                        src = e.param.data.reshape(-1)[a - e.offset:b - e.offset]
                        dst0 = self.shard_off[u] + (a - mine0)
                        self.master[dst0:dst0 + (b - a)].copy_(src)
                for e in self.layout.unit_entries(u):
                    e.param.data = _placeholder(e.shape, self.device)
                    e.param.grad = None
        self.refresh_shadow()
        self.anchor = torch.zeros((), device=self.device, requires_grad=True)
        object.__setattr__(model, "param_store", self)
        self.model = model
        self._full = {}       # unit -> (buffer, work or None)
        self._vec32 = {}      # unit -> {param id: f32 copy of 1-D params}
        self._gfull = {}      # unit -> f32 full-unit gradient buffer
        self._rs = {}         # unit -> [(handle, tmp or None), ...]: reduce-scatters in flight
        self._fresh = set(self.units)  # units whose shard gradient holds no contribution yet
        self._in_backward = False
        self.peak_live_units = 0  # most full-unit buffers (weights + gradients) alive at once
        # --cpu_offload: per-unit pipelined host AdamW (host_step)
        if host:
            from concurrent.futures import ThreadPoolExecutor

            self._copy = torch.cuda.Stream(device=self.device)
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="dpc-host-adamw")
            self._hshadow = (torch.empty(total, dtype=torch.bfloat16, pin_memory=True)
                             if self.compute_dtype == torch.bfloat16 else None)

    # ------------------------------------------------------------------ shards
    def shard(self, flat, u):
        o = self.shard_off[u]
        return flat[o:o + self.shard_len[u]]

    # ------------------------------------------------------------------ host optimizer (offload)
    def host_step(self, opt, grad_scale: float = 1.0) -> None:
        """``--cpu_offload`` AdamW, pipelined per unit: unit u's gradient shard goes D2H on a
        copy stream, a worker thread runs the fused native host AdamW on it
        (``runtime.adamw_host``, OpenMP, GIL released) and queues the H2D upload of its new
        compute copy; the next forward's gather of unit u waits for that unit only, so the
        host update of the later units overlaps the forward of the earlier ones (reference:
        ``CPUOffload(offload_params=True)``, ``/root/reference/main-fsdp.py:60-69``)."""
        opt.step_count += 1
        step = opt.step_count
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._copy.wait_event(ev)
        for u in self.units:
            sl = slice(self.shard_off[u], self.shard_off[u] + self.shard_len[u])
            with torch.cuda.stream(self._copy):
                self.grads_host[sl].copy_(self.grads[sl], non_blocking=True)
                d2h = torch.cuda.Event()
                d2h.record(self._copy)
            self._host_tasks[u] = self._pool.submit(self._host_unit, sl, d2h, opt, step, grad_scale)
        self._d2h_done = torch.cuda.Event()
        self._d2h_done.record(self._copy)

    def _host_unit(self, sl, d2h, opt, step, grad_scale):
        from .. import runtime

        d2h.synchronize()
        b1, b2 = opt.betas
        hs = self._hshadow[sl] if self._hshadow is not None else None
        runtime.adamw_host(self.master[sl], self.grads_host[sl], opt.exp_avg[sl], opt.exp_avg_sq[sl],
                           opt.lr, b1, b2, opt.eps, opt.weight_decay, step, grad_scale, hs)
        with torch.cuda.device(self.device), torch.cuda.stream(self._copy):
            self.shadow[sl].copy_(hs if hs is not None else self.master[sl], non_blocking=True)
            up = torch.cuda.Event()
            up.record(self._copy)
        return up

    def _wait_host(self, u) -> None:
        f = self._host_tasks.pop(u, None)
        if f is not None:
            torch.cuda.current_stream(self.device).wait_event(f.result())

    def wait_host(self) -> None:
        """Every pending host update applied (before reading master / moments / shadow)."""
        for u in list(self._host_tasks):
            self._wait_host(u)

    def refresh_shadow(self):
        self.wait_host()
        src = self.master.to(self.device, non_blocking=True) if self.cpu_offload else self.master
        if self.compute_dtype == torch.float32:
            self.shadow.copy_(src)
        else:
            cast_f32_bf16(src, self.shadow)

    # ------------------------------------------------------------------ gather / release
    def _gather(self, u):
        if u in self._full or not (0 <= u < self.nunits):
            return
        self._wait_host(u)  # --cpu_offload: this unit's updated weights uploaded
        sh = self.shard(self.shadow, u)
        if not self.sharded:
            self._full[u] = (sh, None)  # one rank: the shard is the whole unit
        else:
            buf = torch.empty(self.unit_len[u], dtype=self.compute_dtype, device=self.device)
            self._full[u] = (buf, self.tp.all_gather(buf, sh, async_op=True))
        self._track()

    def _track(self):
        if self.sharded:
            live = len(self._full) + len(self._gfull)
            self.peak_live_units = max(self.peak_live_units, live)

    def _ensure(self, u):
        self._gather(u)
        buf, w = self._full[u]
        if w is not None:
            w.wait()
            self._full[u] = (buf, None)
        return buf

    def _release(self, u):
        self._full.pop(u, None)
        self._vec32.pop(u, None)

    def _rep_view(self, flat, e):
        o = self.rep_off[id(e.param)]
        return flat[o:o + e.numel].view(e.shape)

    def weight(self, p):
        e = self.layout.by_param[id(p)]
        if len(e.shape) < 2:
            return self._rep_view(self.rep_master, e)
        buf = self._full[e.unit][0]
        lo = self.layout.unit_ranges[e.unit][0]
        return buf[e.offset - lo:e.offset - lo + e.numel].view(e.shape)

    def grad(self, p):
        e = self.layout.by_param[id(p)]
        if len(e.shape) < 2:
            return self._rep_view(self.rep_grads, e)
        g = self._gfull[e.unit]
        lo = self.layout.unit_ranges[e.unit][0]
        return g[e.offset - lo:e.offset - lo + e.numel].view(e.shape)

    # ------------------------------------------------------------------ hooks
    def pre_forward(self, u):
        self._ensure(u)
        for k in range(1, self.prefetch + 1):
            self._gather(u + k)

    def post_forward(self, u, training=True):
        last = u == self.nunits - 1
        if not training:
            self._release(u)
        elif self.reshard and not last:
            self._release(u)

    def pre_backward(self, u, need_weights=True):
        self._in_backward = True
        if need_weights:
            self._ensure(u)
            for k in range(1, self.prefetch + 1):
                if u - k >= 1:  # the embeddings unit needs no weights in backward
                    self._gather(u - k)
        if not self.sharded:
            # the weight gradients accumulate straight into the shard (zeroed per step)
            self._gfull[u] = self.shard(self.grads, u)
        else:
            self._gfull[u] = torch.zeros(self.unit_len[u], dtype=torch.float32, device=self.device)
        self._track()

    def post_backward(self, u):
        self._release(u)
        g = self._gfull.pop(u)
        if not self.sharded:
            return
        out = self.shard(self.grads, u)
        if self.reduce_dtype != torch.float32:
            g = g.to(self.reduce_dtype)
            tmp = torch.empty(self.shard_len[u], dtype=self.reduce_dtype, device=self.device)
            rs = (self.tp.reduce_scatter(tmp, g, async_op=True), tmp)
        elif u in self._fresh:
            # first contribution since zero_grad: reduce-scatter straight into the shard
            rs = (self.tp.reduce_scatter(out, g, async_op=True), None)
        else:
            tmp = torch.empty(self.shard_len[u], dtype=torch.float32, device=self.device)
            rs = (self.tp.reduce_scatter(tmp, g, async_op=True), tmp)
        # (a list: a unit whose backward runs twice in a step has two in flight, both waited)
        self._rs.setdefault(u, []).append(rs)
        self._fresh.discard(u)
        # g is dropped here: the transport keeps it alive until the collective has read it

    def finish_grads(self):
        rep_w = None
        if self.sharded:
            rep_w = self.tp.all_reduce(self.rep_grads, async_op=True)
        for u, lst in sorted(self._rs.items()):
            for w, tmp in lst:
                w.wait()
                if tmp is not None:
                    self.shard(self.grads, u).add_(tmp.float())
        self._rs.clear()
        if rep_w is not None:
            rep_w.wait()
        self._in_backward = False
        # anything still gathered from the forward (e.g. the head) is released now
        for u in list(self._full):
            self._release(u)

    def finish_grads_and_update(self, opt, opt_rep, grad_scale: float = 1.0):
        """``finish_grads`` + both AdamW steps, unit by unit: each unit's shard is updated as
        soon as its reduce-scatter has landed (units complete in backward order, the last
        layer's first), while the earlier units' reduce-scatters are still on the comm stream --
        as the DDP engine does bucket by bucket.  Only the last units' reduce-scatters remain on
        the critical path.  Same arithmetic as ``finish_grads`` then ``opt.step`` (AdamW is
        element-wise; the step count advances once)."""
        rep_w = self.tp.all_reduce(self.rep_grads, async_op=True) if self.sharded else None
        opt.begin_step()
        done = set()
        for u in sorted(self._rs, reverse=True):  # (reduce-scatters were issued last unit first)
            for w, tmp in self._rs[u]:
                with mark("comm:wait_unit"):
                    w.wait()
                if tmp is not None:
                    self.shard(self.grads, u).add_(tmp.float())
            lo = self.shard_off[u]
            opt.update(lo, lo + self.shard_len[u], grad_scale=grad_scale)
            done.add(u)
        for u in self.units:  # (a unit without a reduce-scatter this step: one rank, or no grad)
            if u not in done:
                lo = self.shard_off[u]
                opt.update(lo, lo + self.shard_len[u], grad_scale=grad_scale)
        self._rs.clear()
        if rep_w is not None:
            rep_w.wait()
        opt_rep.step(grad_scale=grad_scale)
        self._in_backward = False
        for u in list(self._full):
            self._release(u)

    def reset_step_state(self):
        """After a failed HIP-graph capture: no gathered unit, gradient buffer or
        reduce-scatter the capture recorded exists (engine/base.py:Engine.reset_step_state)."""
        self._full.clear()
        self._vec32.clear()
        self._gfull.clear()
        self._rs.clear()
        self._fresh = set(self.units)
        self._in_backward = False

    def zero_grad(self):
        if self._d2h_done is not None:  # the host optimizer's gradient copies read grads first
            torch.cuda.current_stream(self.device).wait_event(self._d2h_done)
            self._d2h_done = None
        self.grads.zero_()
        self.rep_grads.zero_()
        self._fresh = set(self.units)

    # ------------------------------------------------------------------ full state
    @torch.no_grad()
    def gather_full(self, flat_shards, dst_rank: int = 0, dtype=torch.float32, rep_flat=None):
        """Canonical {name: tensor} of a sharded flat f32 buffer (params or optimizer
        moments), materialised on ``dst_rank`` (others return None).  Collective.
        ``rep_flat``: the replicated buffer holding the 1-D entries (default: rep_master)."""
        self.wait_host()
        rep_flat = self.rep_master if rep_flat is None else rep_flat
        out = {} if self.rank == dst_rank else None
        for u in self.units:
            sh = self.shard(flat_shards, u).to(self.device).contiguous()
            if not self.sharded:
                full = sh
            elif not getattr(self.tp, "p2p", True):  # (a transport without point-to-point: all-gather)
                full = torch.empty(self.unit_len[u], dtype=sh.dtype, device=self.device)
                self.tp.all_gather(full, sh)
                if self.rank != dst_rank:
                    continue
            elif self.rank == dst_rank:
                # gathered to dst_rank ONLY (grouped point-to-point): the reference's
                # FULL_STATE_DICT all-gathers every unit onto every rank (main-fsdp.py:193-194),
                # W x the traffic a rank-0 checkpoint needs
                L = self.shard_len[u]
                full = torch.empty(self.unit_len[u], dtype=sh.dtype, device=self.device)
                full[self.rank * L:(self.rank + 1) * L].copy_(sh)
                self.tp.sendrecv(recvs=[(full[r * L:(r + 1) * L], r) for r in range(self.tp.size) if r != dst_rank])
            else:
                self.tp.sendrecv(sends=[(sh, dst_rank)])
                continue
            if out is not None:
                lo = self.layout.unit_ranges[u][0]
                for e in self.layout.unit_entries(u):
                    src = (self._rep_view(rep_flat, e) if len(e.shape) < 2 else
                           full[e.offset - lo:e.offset - lo + e.numel].view(e.shape))
                    out[e.name] = src.to("cpu", dtype=dtype, copy=True)
        return out

    @torch.no_grad()
    def load_full(self, sd: dict, flat_shards, rep_flat=None):
        rep_flat = self.rep_master if rep_flat is None else rep_flat
        for e in self.rep:
            self._rep_view(rep_flat, e).copy_(sd[e.name].reshape(e.shape))
        for u in self.units:
            lo = self.layout.unit_ranges[u][0]
            mine0 = lo + self.rank * self.shard_len[u]
            mine1 = mine0 + self.shard_len[u]
            for e in self.layout.unit_entries(u):
                a, b = max(e.offset, mine0), min(e.offset + e.numel, mine1)
                if a < b:
                    src = sd[e.name].reshape(-1)[a - e.offset:b - e.offset]
                    dst0 = self.shard_off[u] + (a - mine0)
                    flat_shards[dst0:dst0 + (b - a)].copy_(src)
