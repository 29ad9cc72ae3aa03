"""Pipeline (and pipeline x data parallel) engine: recipes ``main-pipe.py`` and
``main-pipe-ddp.py``.

Reference: ``/root/reference/main-pipe.py:85-221`` (GPipe via torch Pipe, chunks =
stages, single process) and ``main-pipe-ddp.py`` (an empty stub).  Here: one process per
GPU on a (pp, dp) mesh -- rank = stage * dp + replica -- each stage owning a contiguous,
cost-balanced run of units (``parallel/pipeline.py``), micro-batches (default 4 x stages)
executed in exactly the order ``schedule_1f1b`` (default), ``schedule_gpipe`` or the zero-bubble
``schedule_zb`` (backward split into B and deferred W passes: ``models/fused.py:defer_weight_grads``) gives,
activations exchanged by asynchronous grouped RCCL send/recv between neighbouring stages
(``run_schedule``; optional bf16 wire format), and, for dp > 1, each stage's gradients
all-reduced across its replicas with the bucketed DDP store once the last micro-batch's
backward has produced them.  The pipeline and replica communicators are ONE native RCCL
communicator split with ncclCommSplit (``parallel/transport.py``).

The loss is the exact mean over all valid tokens of the batch: micro-batch losses are
weighted by their share of valid targets (computed on device, no sync).
"""
from __future__ import annotations

from contextlib import nullcontext as _nullcontext

import torch
import torch.distributed as dist

from ..models.fused import defer_weight_grads, run_embeddings, run_head, run_layers
from ..ops.optim import FlatAdamW
from ..parallel import comm
from ..parallel.ddp import DDPStore
from ..parallel.fsdp import _placeholder
from ..parallel.pipeline import (P2P, partition, run_schedule, schedule_1f1b, schedule_gpipe, schedule_zb,
                                 stage_costs, unit_costs)
from ..parallel.store import LocalStore
from ..parallel.transport import TorchTransport, make_mesh_transports
from ..parallel.transport import check_drained
from ..utils.profiling import mark
from .base import Engine, GraphedStep


class PipelineEngine(Engine):
    name = "pipe"
    collective_generate = True

    def __init__(self, model, device, lr: float, pp: int, dp: int = 1, num_microbatches: int = 0,
                 schedule: str = "1f1b", bucket_mb: float = 128.0, compute_dtype=None,
                 seq_len: int | None = None, grad_scaler: bool = False, comm_kind: str | None = None,
                 wire_dtype=None, graph: bool = False, force_dist: bool = False,
                 reduce_dtype=torch.float32):
        self.device = torch.device(device)
        self.model = model
        if grad_scaler:
            from ..ops.amp import GradScaler

            self.scaler = GradScaler(self.device)
        world = comm.world_size()
        if pp * dp != world:
            raise ValueError(f"pp ({pp}) x dp ({dp}) must equal the world size ({world})")
        self.pp, self.dp = pp, dp
        if world > 1:
            self.pp_group, self.dp_group, self.stage, self.replica, pp_ranks = comm.make_mesh(pp, dp)
            self.pp_tp, self.dp_tp = make_mesh_transports(self.pp_group, self.dp_group, self.stage,
                                                          self.replica, self.device, comm_kind)
        elif force_dist:
            # one rank on the N > 1 path (bench.py --force_dist_path): the replica store is the
            # bucketed DDP store over a native 1-rank communicator (no neighbour: no p2p)
            from ..parallel.transport import make_transport

            self.pp_group = self.dp_group = None
            self.stage, self.replica, pp_ranks = 0, 0, [0]
            self.pp_tp = TorchTransport(None)
            self.dp_tp = make_transport(None, self.device, "native")
        else:
            self.pp_group = self.dp_group = None
            self.stage, self.replica, pp_ranks = 0, 0, [0]
            self.pp_tp = self.dp_tp = TorchTransport(None)
        self.dp_world = dp
        self.dp_rank = self.replica
        self.first = self.stage == 0
        self.last = self.stage == pp - 1
        self.is_logger = comm.rank() == 0
        # micro-batches: by default the largest divisor of the per-replica batch that is at most
        # 4 x stages (the 1F1B bubble is (pp - 1) / (M + pp - 1): 18 % at pp 8, M 32); one stage
        # has no bubble to hide, so it runs the whole batch at once (the reference: chunks =
        # num_stages, /root/reference/main-pipe.py:83).  The batch size is known at the first
        # step (_micro_count).
        self.n_micro_req = num_microbatches
        self.schedule = schedule
        # (the zero-bubble schedules leave less bubble to amortise: 2 x stages micro-batches --
        # larger ones, a smaller per-micro-batch tax; bench/pp_stage_proxy.py, profiles/r6_pp/)
        self._mfac = 2 if schedule in ("zb", "zb2") else 4
        self.n_micro = max(1, num_microbatches or (self._mfac * pp if pp > 1 else 1))
        S = seq_len or model.max_position_embeddings
        groups = partition(unit_costs(model, S), pp)
        self.groups = groups
        self.my_units = groups[self.stage]
        nunits = model.num_layers + 2
        self.layers = [model.decoder.layers[u - 1] for u in self.my_units if 1 <= u <= model.num_layers]
        # free parameters of units owned by other stages before building the store
        mine = set(self.my_units)
        for ui, (_, mods) in enumerate(model.units()):
            if ui not in mine:
                for mod in mods:
                    for p in mod.parameters():
                        p.data = _placeholder(p.shape, self.device)
        if dp > 1 or force_dist:
            self.store = DDPStore(model, device, group=self.dp_group, bucket_mb=bucket_mb,
                                  reduce_dtype=reduce_dtype, compute_dtype=compute_dtype,
                                  units=self.my_units, transport=self.dp_tp)
        else:
            self.store = LocalStore(model, device, compute_dtype=compute_dtype, units=self.my_units)
        self.store.accum_steps = self.n_micro
        self.opt = FlatAdamW(self.store.master, self.store.grads, lr=lr, shadow=self.store.shadow)
        self.p2p = P2P(self.pp_tp, self.stage, pp, self.device, wire_dtype=wire_dtype)
        self.pp_ranks = pp_ranks
        self.D = model.dim
        assert nunits == len(model.units())
        if world > 1:
            # bring up the communicators before the first (grouped) p2p
            t = torch.zeros(1, device=self.device)
            self.pp_tp.all_reduce(t)
            self.dp_tp.all_reduce(t)
        # HIP-graph "compile": the whole step -- every micro-batch's forward / backward, the
        # asynchronous p2p and the replica all-reduces -- as one graph (single stage, or
        # capturable native transports)
        self.graph = graph and self.device.type == "cuda" and (
            world == 1 or (self.pp_tp.capturable() and (dp == 1 or self.dp_tp.capturable())))
        self._stepper = GraphedStep(self, [self.opt])
        self._cost_cache = {}

    # ------------------------------------------------------------------ pieces
    def _micro_count(self, N: int) -> int:
        if self.n_micro_req:
            return self.n_micro_req
        if self.pp == 1:
            return 1
        mfac = getattr(self, "_mfac", 4)
        return max(d for d in range(1, min(N, mfac * self.pp) + 1) if N % d == 0)

    def _split(self, batch, targets):
        N = batch["input_ids"].shape[0]
        M = self.n_micro = self._micro_count(N)
        self.store.accum_steps = M
        if N % M:
            raise ValueError(f"batch {N} not divisible by {M} micro-batches")
        mb = N // M
        out = []
        for m in range(M):
            sl = slice(m * mb, (m + 1) * mb)
            out.append((batch["input_ids"][sl], batch["position_ids"][sl],
                        None if batch.get("mask") is None else batch["mask"][sl],
                        targets[sl] if targets is not None else None))
        return out, mb

    def _fwd(self, mbatch, x_in, training, want_correct=False):
        ids, pos, mask, tg = mbatch
        mb, S = ids.shape
        st = self.store
        if mask is not None:
            mask = mask.to(torch.bool).contiguous()
        if self.first:
            x = run_embeddings(self.model, st, ids, pos, training)
        else:
            x = x_in
        x = run_layers(self.model, st, x, mask, mb, S, self.layers, training, head_next=self.last)
        if self.last:
            return run_head(self.model, st, x, tg, training, want_correct)
        return x

    def _act_shape(self, mb, S):
        return (mb * S, self.D)

    # ------------------------------------------------------------------ training
    def train_step(self, batch, targets):
        out = self._stepper(self._step_body, batch, targets) if self.graph else self._step_body(batch, targets)
        check_drained(f"the end of a {self.name} step")  # --stream_check
        return out

    def _step_body(self, batch, targets):
        st = self.store
        st.zero_grad()
        micro, mb = self._split(batch, targets)
        S = batch["input_ids"].shape[1]
        shape = self._act_shape(mb, S)
        n_total = (targets != -100).sum().float().clamp_min(1.0) if self.last else None
        inputs, outputs = {}, {}
        acc = {"loss": torch.zeros((), device=self.device)} if self.last else {}

        def forward(m, x):
            if x is not None:
                x.requires_grad_(True)
            with mark(f"fwd mb{m}"):
                out = self._fwd(micro[m], x, True)
            inputs[m] = x
            if self.last:
                loss, n_valid, _ = out
                w = n_valid / n_total
                outputs[m] = loss * w
                acc["loss"] = acc["loss"] + (loss * w).detach()
                return None
            outputs[m] = out
            return out

        zb = self.schedule in ("zb", "zb2")
        wq = {}  # zero-bubble: micro-batch -> its deferred weight-gradient closures

        def backward(m, g):
            y = outputs.pop(m)
            with mark(f"bwd mb{m}"):
                with defer_weight_grads(wq.setdefault(m, [])) if zb else _nullcontext():
                    if self.last:
                        self._scaled(y).backward()
                    else:
                        torch.autograd.backward(y, g)
            x = inputs.pop(m)
            return None if x is None else x.grad

        def wgrad(m):
            with mark(f"wgrad mb{m}"):
                for fn in wq.pop(m):
                    fn()

        if zb:
            order = schedule_zb(self.n_micro, self.stage, self.pp, costs=self._zb_costs(S),
                                mem=2 if self.schedule == "zb2" else 1)
        else:
            order = (schedule_gpipe if self.schedule == "gpipe" else schedule_1f1b)(self.n_micro, self.stage, self.pp)
        run_schedule(order, self.first, self.last, forward, backward, self.p2p, shape, wgrad=wgrad)
        assert not wq, "zero-bubble schedule left weight gradients unrun"
        if isinstance(st, DDPStore) and st.tp.active and self.scaler is None:
            # bucket by bucket, as the DDP engine does: AdamW of the buckets whose replica
            # all-reduce has landed runs while the later ones are still on the links (a stage's
            # buckets launch from its last micro-batch's backward -- or W -- passes, unit by unit)
            with mark("optim"):
                st.launch_all()
                self.opt.begin_step()
                for bi in range(len(st.buckets)):
                    with mark("comm:wait_bucket"):
                        st.wait_bucket(bi)
                    lo, hi = st.bucket_range(bi)
                    self.opt.update(lo, hi, grad_scale=1.0 / self.dp)
                st.reset_buckets()
            return acc.get("loss")
        if isinstance(st, DDPStore):
            with mark("comm:finish_grads"):
                st.finish_grads()
        with mark("optim"):
            return self._optim(acc)

    def _zb_costs(self, S):
        """Per-stage (F, B, W) costs of the zero-bubble simulation: the same on every rank (model
        configuration, sequence length and partition only)."""
        key = ("zb", S)
        if self._cost_cache.get(key) is None:
            self._cost_cache[key] = tuple(stage_costs(self.model, S, self.groups))
        return self._cost_cache[key]

    def _optim(self, acc):
        if self.scaler is not None:
            # every stage holds different gradients: one skip decision for the whole job
            self.scaler.check(self.opt.grad)
            self.scaler.reduce_flag(None)
            self.opt.step(grad_scale=1.0 / self.dp, **self.scaler.opt_kwargs(self.opt))
            self.scaler.update()
            return acc.get("loss")
        self.opt.step(grad_scale=1.0 / self.dp)
        return acc.get("loss")

    @torch.no_grad()
    def eval_step(self, batch, targets):
        micro, mb = self._split(batch, targets)
        S = batch["input_ids"].shape[1]
        shape = self._act_shape(mb, S)
        tot = [torch.zeros((), device=self.device) for _ in range(3)]
        for m in range(self.n_micro):
            x, _ = self.p2p.exchange(recv_prev_shape=None if self.first else shape)
            out = self._fwd(micro[m], x, False, want_correct=True)
            if self.last:
                loss, n_valid, n_corr = out
                tot[0] = tot[0] + loss * n_valid
                tot[1] = tot[1] + n_valid
                tot[2] = tot[2] + n_corr
            else:
                self.p2p.exchange(send_next=out)
        return tot if self.last else None

    # ------------------------------------------------------------------ generation
    def lm(self):
        eng = self

        @torch.no_grad()
        def forward(input_ids, position_ids, mask=None):
            from ..models.fused import head_logits, last_rows

            N, S = input_ids.shape
            shape = (N * S, eng.D)
            x, _ = eng.p2p.exchange(recv_prev_shape=None if eng.first else shape)
            st = eng.store
            if eng.first:
                x = run_embeddings(eng.model, st, input_ids, position_ids, False)
            x = run_layers(eng.model, st, x, None, N, S, eng.layers, False)  # (output formed here)
            V = eng.model.vocab_size
            tok = torch.zeros(1, dtype=torch.int64, device=eng.device)
            if eng.last:
                tok[0] = head_logits(eng.model, last_rows(x, N, S), st)[0].argmax()
            else:
                eng.p2p.exchange(send_next=x)
            if eng.pp > 1:
                eng.pp_tp.broadcast(tok, src=eng.pp - 1)
            out = torch.zeros(1, 1, V, device=eng.device)
            out[0, 0, tok[0]] = 1.0
            return out

        forward.max_position_embeddings = self.model.max_position_embeddings
        return forward

    # ------------------------------------------------------------------ state
    def _gather_named(self, named: dict):
        """Merge per-stage {name: cpu tensor} dicts onto global rank 0 (replica 0 only)."""
        if self.pp == 1:
            return named if self.is_logger else None
        if self.replica != 0:
            return None
        objs = [None] * self.pp if self.stage == 0 else None
        dist.gather_object(named, objs, dst=self.pp_ranks[0], group=self.pp_group)
        if self.stage != 0:
            return None
        merged = {}
        for o in objs:
            merged.update(o)
        # canonical order
        order = [n for n, _ in self.model.named_parameters()]
        return {k: merged[k] for k in order if k in merged}

    def _named_flat(self, flat):
        return {e.name: self.store._view(flat, e).detach().to("cpu", copy=True) for e in self.store.entries}

    def full_state_dict(self):
        return self._gather_named(self._named_flat(self.store.master))

    def load_model_state(self, sd):
        self.store.load_state_dict(sd, strict=False)

    def train_state(self):
        m = self._gather_named(self._named_flat(self.opt.exp_avg))
        v = self._gather_named(self._named_flat(self.opt.exp_avg_sq))
        return {"optimizer": {"step": self.opt.step_count, "exp_avg": m, "exp_avg_sq": v,
                              "format": "canonical"}, **self._scaler_state()}

    def load_train_state(self, st):
        o = st["optimizer"]
        self.opt.step_count = int(o["step"])
        for key, flat in (("exp_avg", self.opt.exp_avg), ("exp_avg_sq", self.opt.exp_avg_sq)):
            d = o.get(key)
            if isinstance(d, dict):
                for e in self.store.entries:
                    if e.name in d:
                        self.store._view(flat, e).copy_(d[e.name])
        self._load_scaler_state(st)

    @property
    def step_count(self):
        return self.opt.step_count
