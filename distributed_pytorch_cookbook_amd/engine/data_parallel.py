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
from .base import Engine


class DataParallelEngine(Engine):
    name = "ddp"

    def __init__(self, model, device, lr: float, group=None, bucket_mb: float = 128.0,
                 reduce_dtype=torch.float32, overlap: bool = True, compute_dtype=None,
                 graph: bool = False, native_comm: bool = False, grad_scaler: bool = False):
        self.device = torch.device(device)
        self.model = model
        self.dp_group = group
        self.dp_world = comm.world_size(group)
        self.dp_rank = comm.rank(group)
        self.is_logger = comm.rank() == 0
        if self.dp_world > 1:
            self.store = DDPStore(model, device, group=group, bucket_mb=bucket_mb,
                                  reduce_dtype=reduce_dtype, overlap=overlap, compute_dtype=compute_dtype,
                                  native=native_comm)
        else:
            self.store = LocalStore(model, device, compute_dtype=compute_dtype)
        self.opt = FlatAdamW(self.store.master, self.store.grads, lr=lr, shadow=self.store.shadow)
        if grad_scaler:
            from ..ops.amp import GradScaler

            self.scaler = GradScaler(self.device)
        self.graph = graph and self.device.type == "cuda" and self.dp_world == 1
        self._graph = None
        self._gkey = None

    # ------------------------------------------------------------------ training
    def _step_body(self, batch, targets):
        self.store.zero_grad()
        out = self.model(**batch, targets=targets)
        self._scaled(out.loss).backward()
        if self.scaler is not None:
            # the non-finite check needs every bucket reduced before any parameter moves;
            # all-reduced gradients are identical on every rank, so is the flag
            if self.dp_world > 1:
                self.store.finish_grads()
            self.scaler.check(self.store.grads)
            self.opt.step(grad_scale=1.0 / self.dp_world, **self.scaler.opt_kwargs(self.opt))
            self.scaler.update()
            return out.loss.detach()
        if self.dp_world > 1 and self.store.master.is_cuda:
            # bucket by bucket: AdamW of the buckets already reduced runs on the compute stream
            # while the last ones (the embeddings, whose backward comes last) are still being
            # all-reduced on the comm stream
            st = self.store
            st.launch_all()
            self.opt.begin_step()
            for bi in range(len(st.buckets)):
                st.wait_bucket(bi)
                lo, hi = st.bucket_range(bi)
                self.opt.update(lo, hi, grad_scale=1.0 / self.dp_world)
            st.reset_buckets()
            return out.loss.detach()
        if self.dp_world > 1:
            self.store.finish_grads()
        self.opt.step(grad_scale=1.0 / self.dp_world)
        return out.loss.detach()

    def train_step(self, batch, targets):
        if not self.graph:
            return self._step_body(batch, targets)
        return self._graph_step(batch, targets)

    def _graph_step(self, batch, targets):
        """The whole step (memset of the grads, forward, backward, AdamW) as ONE HIP graph.

        Call 1 for a given input signature runs eagerly (lazy init, allocator warm-up), call 2
        captures the step into a graph against static input buffers and replays it, later
        calls copy the batch into the static buffers and replay.  AdamW reads its step count
        from a device counter, so replays apply the right bias corrections."""
        mask = batch.get("mask")
        key = (tuple(batch["input_ids"].shape), mask is None)
        if self._graph is not None and key == self._gkey:
            self._static["ids"].copy_(batch["input_ids"], non_blocking=True)
            self._static["pos"].copy_(batch["position_ids"], non_blocking=True)
            self._static["tg"].copy_(targets, non_blocking=True)
            if mask is not None:
                self._static["mask"].copy_(mask, non_blocking=True)
            self._graph.replay()
            self.opt.step_count += 1
            return self._static_loss.clone()
        if self._gkey != key:  # first call for this signature: eager (warm-up)
            self._gkey = key
            self._graph = None
            return self._step_body(batch, targets)
        st = {"ids": batch["input_ids"].clone(), "pos": batch["position_ids"].clone(),
              "tg": targets.clone(), "mask": None if mask is None else mask.clone()}
        self._static = st
        self.opt.device_step = True
        g = torch.cuda.CUDAGraph()
        torch.cuda.synchronize()
        try:
            with torch.cuda.graph(g):
                b = {"input_ids": st["ids"], "position_ids": st["pos"], "mask": st["mask"]}
                self._static_loss = self._step_body(b, st["tg"])
        except Exception as exc:  # capture not possible: stay eager
            self.opt.device_step = False
            self.graph = False
            if self.is_logger:
                print(f"[hip-graph] capture failed ({exc!r}); running eagerly")
            return self._step_body(batch, targets)
        self._graph = g
        self._graph.replay()
        return self._static_loss.clone()

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
