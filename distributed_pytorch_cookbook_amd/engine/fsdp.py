"""FSDP engine (recipe ``main-fsdp.py``): sharded store + sharded AdamW.

Reference: ``/root/reference/main-fsdp.py:42-202``.  Differences by design: generation
runs on every rank (the reference ran it on rank 0 only through an FSDP module, an
unmatched-collective hang, ``main-fsdp.py:184-188``); the final state dict is gathered
unit by unit to rank 0 only instead of materialising the full model on every GPU
(``main-fsdp.py:194``).
"""
from __future__ import annotations

import os

import torch

from ..ops.optim import FlatAdamW
from ..parallel import comm
from ..parallel.fsdp import FSDPStore
from ..parallel.transport import check_drained
from ..utils.profiling import mark
from .base import Engine, GraphedStep

# A/B switch (bench/offload.py): the synchronous offload step (D2H, host AdamW, H2D in turn)
_OFFLOAD_SYNC = os.environ.get("DPC_OFFLOAD_SYNC", "0") == "1"


class FSDPEngine(Engine):
    name = "fsdp"
    collective_generate = True

    def __init__(self, model, device, lr: float, group=None, prefetch: int = 1,
                 reshard_after_forward: bool = True, cpu_offload: bool = False, compute_dtype=None,
                 reduce_dtype=torch.float32, grad_scaler: bool = False, graph: bool = False,
                 comm_kind: str | None = None, force_sharded: bool = False):
        self.device = torch.device(device)
        self.model = model
        self.dp_group = group
        self.dp_world = comm.world_size(group)
        self.dp_rank = comm.rank(group)
        self.is_logger = comm.rank() == 0
        self.store = FSDPStore(model, device, group=group, compute_dtype=compute_dtype,
                               prefetch=prefetch, reshard_after_forward=reshard_after_forward,
                               cpu_offload=cpu_offload, reduce_dtype=reduce_dtype, comm_kind=comm_kind,
                               force_sharded=force_sharded)
        st = self.store
        grad = st.grads_host if st.cpu_offload else st.grads
        self.opt = FlatAdamW(st.master, grad, lr=lr, shadow=st.shadow)
        self.opt_rep = FlatAdamW(st.rep_master, st.rep_grads, lr=lr)  # replicated 1-D params
        if grad_scaler:
            from ..ops.amp import GradScaler

            self.scaler = GradScaler(self.device)
        # HIP-graph "compile" of the whole sharded step (gathers, reduce-scatters, AdamW);
        # not with --cpu_offload, whose optimizer runs on the host
        self.graph = (graph and self.device.type == "cuda" and not st.cpu_offload
                      and (not st.sharded or st.tp.capturable()))
        self._stepper = GraphedStep(self, [self.opt, self.opt_rep])

    def train_step(self, batch, targets):
        out = self._stepper(self._step_body, batch, targets) if self.graph else self._step_body(batch, targets)
        check_drained(f"the end of a {self.name} step")  # --stream_check
        return out

    def _step_body(self, batch, targets):
        st = self.store
        st.zero_grad()
        with mark("fwd"):  # (unit all-gathers enqueued inside: "comm:all_gather")
            out = self.model(**batch, targets=targets)
        with mark("bwd"):  # (re-gathers and reduce-scatters enqueued inside)
            self._scaled(out.loss).backward()
        if self.scaler is None and not st.cpu_offload and st.sharded and st.tp.active:
            # unit by unit: AdamW of the units already reduce-scattered on the compute stream
            # while the remaining reduce-scatters are still on the comm stream
            with mark("optim"):
                st.finish_grads_and_update(self.opt, self.opt_rep, grad_scale=1.0 / self.dp_world)
            return out.loss.detach()
        with mark("comm:finish_grads"):
            st.finish_grads()
        with mark("optim"):
            return self._optim(out)

    def _optim(self, out):
        st = self.store
        if st.cpu_offload and self.scaler is None and not _OFFLOAD_SYNC:
            # pipelined host AdamW: overlaps the next step's forward (FSDPStore.host_step)
            st.host_step(self.opt, grad_scale=1.0 / self.dp_world)
            self.opt_rep.step(grad_scale=1.0 / self.dp_world)
            return out.loss.detach()
        if st.cpu_offload:
            st.grads_host.copy_(st.grads, non_blocking=True)
            torch.cuda.current_stream().synchronize()  # grads_host D2H landed
        if self.scaler is not None:
            # shards differ per rank: the skip decision is reduced over the group
            sc = self.scaler
            sc.check(self.opt.grad)
            sc.check(self.opt_rep.grad)
            sc.reduce_flag(self.dp_group)
            self.opt.step(grad_scale=1.0 / self.dp_world, **sc.opt_kwargs(self.opt))
            self.opt_rep.step(grad_scale=1.0 / self.dp_world, **sc.opt_kwargs(self.opt_rep))
            sc.update()
            return out.loss.detach()
        self.opt.step(grad_scale=1.0 / self.dp_world)
        self.opt_rep.step(grad_scale=1.0 / self.dp_world)
        return out.loss.detach()

    @torch.no_grad()
    def eval_step(self, batch, targets):
        out = self.model(**batch, targets=targets, want_correct=True)
        return out.loss * out.n_valid, out.n_valid, out.n_correct

    def lm(self):
        return self.model

    def full_state_dict(self):
        return self.store.gather_full(self.store.master, dst_rank=0)

    def load_model_state(self, sd):
        self.store.wait_host()
        self.store.load_full(sd, self.store.master)
        self.store.refresh_shadow()

    def train_state(self):
        st = self.store
        m = st.gather_full(self.opt.exp_avg, dst_rank=0, rep_flat=self.opt_rep.exp_avg)
        v = st.gather_full(self.opt.exp_avg_sq, dst_rank=0, rep_flat=self.opt_rep.exp_avg_sq)
        return {"optimizer": {"step": self.opt.step_count, "exp_avg": m, "exp_avg_sq": v,
                              "format": "canonical"}, **self._scaler_state()}

    def load_train_state(self, st):
        self.store.wait_host()
        o = st["optimizer"]
        self.opt.step_count = int(o["step"])
        self.opt_rep.step_count = int(o["step"])
        if isinstance(o.get("exp_avg"), dict):
            self.store.load_full(o["exp_avg"], self.opt.exp_avg, rep_flat=self.opt_rep.exp_avg)
            self.store.load_full(o["exp_avg_sq"], self.opt.exp_avg_sq, rep_flat=self.opt_rep.exp_avg_sq)
        self._load_scaler_state(st)

    @property
    def step_count(self):
        return self.opt.step_count
