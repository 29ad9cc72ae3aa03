"""Single-device and data-parallel engines (recipes ``main-single.py`` / ``main-ddp.py``).

Reference step (``/root/reference/main-single.py:85-101``, ``main-ddp.py:110-126``):
zero_grad -> autocast forward -> cross-entropy -> GradScaler backward -> step.  Here:
memset of the flat gradient buffer -> fused forward with the loss inside the head ->
backward (DDP bucket all-reduces fire from inside it) -> wait for the last buckets ->
one fused AdamW launch (which also folds in the 1/W average and refreshes the bf16
weights).  No GradScaler: bf16 needs none.  With ``graph=True`` the
whole single-GPU step is captured once into a HIP graph and replayed (the cookbook's
meaning of "compile", replacing torch.compile/Inductor).
"""
from __future__ import annotations

import torch

from ..ops.optim import FlatAdamW
from ..parallel import comm
from ..parallel.ddp import DDPStore
from ..parallel.store import LocalStore
from ..parallel.transport import check_drained
from ..utils.profiling import mark
from .base import Engine, GraphedStep


class DataParallelEngine(Engine):
    name = "ddp"

    def __init__(self, model, device, lr: float, group=None, bucket_mb: float = 128.0,
                 reduce_dtype=torch.float32, overlap: bool = True, compute_dtype=None,
                 graph: bool = False, comm_kind: str | None = None, grad_scaler: bool = False,
                 force_ddp_store: bool = False):
        self.device = torch.device(device)
        self.model = model
        self.dp_group = group
        self.dp_world = comm.world_size(group)
        self.dp_rank = comm.rank(group)
        self.is_logger = comm.rank() == 0
        if self.dp_world > 1 or force_ddp_store:
            # (force_ddp_store: the bucketed store and its transport at one rank -- tests)
            self.store = DDPStore(model, device, group=group, bucket_mb=bucket_mb,
                                  reduce_dtype=reduce_dtype, overlap=overlap, compute_dtype=compute_dtype,
                                  comm_kind=comm_kind)
        else:
            self.store = LocalStore(model, device, compute_dtype=compute_dtype)
        self.opt = FlatAdamW(self.store.master, self.store.grads, lr=lr, shadow=self.store.shadow)
        if grad_scaler:
            from ..ops.amp import GradScaler

            self.scaler = GradScaler(self.device)
        # HIP-graph "compile": at one rank, or across ranks when the gradient all-reduces ride
        # the capturable native RCCL transport
        tp = getattr(self.store, "tp", None)
        self.graph = graph and self.device.type == "cuda" and (self.dp_world == 1 or (tp is not None and tp.capturable()))
        self._stepper = GraphedStep(self, [self.opt])

    # ------------------------------------------------------------------ training
    def _step_body(self, batch, targets):
        self.store.zero_grad()
        with mark("fwd"):
            out = self.model(**batch, targets=targets)
        with mark("bwd"):  # (the DDP bucket all-reduces are enqueued from inside it: "comm:*")
            self._scaled(out.loss).backward()
        with mark("optim"):
            return self._optim(out)

    def _optim(self, out):
        if self.scaler is not None:
            # the non-finite check needs every bucket reduced before any parameter moves;
            # all-reduced gradients are identical on every rank, so is the flag
            if isinstance(self.store, DDPStore):
                self.store.finish_grads()
            self.scaler.check(self.store.grads)
            self.opt.step(grad_scale=1.0 / self.dp_world, **self.scaler.opt_kwargs(self.opt))
            self.scaler.update()
            return out.loss.detach()
        if isinstance(self.store, DDPStore) and self.store.tp.active and self.store.master.is_cuda:
            # bucket by bucket: AdamW of the buckets already reduced runs on the compute stream
            # while the last ones (the embeddings, whose backward comes last) are still being
            # all-reduced on the comm stream
            st = self.store
            st.launch_all()
            self.opt.begin_step()
            for bi in range(len(st.buckets)):
                with mark("comm:wait_bucket"):
                    st.wait_bucket(bi)
                lo, hi = st.bucket_range(bi)
                self.opt.update(lo, hi, grad_scale=1.0 / self.dp_world)
            st.reset_buckets()
            return out.loss.detach()
        if isinstance(self.store, DDPStore):
            self.store.finish_grads()
        self.opt.step(grad_scale=1.0 / self.dp_world)
        return out.loss.detach()

    def train_step(self, batch, targets):
        out = self._stepper(self._step_body, batch, targets) if self.graph else self._step_body(batch, targets)
        check_drained(f"the end of a {self.name} step")  # --stream_check
        return out

    @torch.no_grad()
    def eval_step(self, batch, targets):
        out = self.model(**batch, targets=targets, want_correct=True)
        return out.loss * out.n_valid, out.n_valid, out.n_correct

    def lm(self):
        return self.model

    # ------------------------------------------------------------------ state
    def full_state_dict(self):
        return self.store.state_dict()

    def load_model_state(self, sd):
        self.store.load_state_dict(sd)

    def train_state(self):
        return {"optimizer": {k: (v.detach().cpu() if torch.is_tensor(v) else v)
                              for k, v in self.opt.state_dict().items()}, **self._scaler_state()}

    def load_train_state(self, st):
        self.opt.load_state_dict({k: (v.to(self.device) if torch.is_tensor(v) else v)
                                  for k, v in st["optimizer"].items()})
        self._load_scaler_state(st)

    @property
    def step_count(self):
        return self.opt.step_count
