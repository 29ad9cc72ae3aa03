"""Engine interface: what a recipe's training loop needs from a parallelism strategy.

The reference's recipes differ only in the wrapper around the model (SURVEY.md §1,
observation 2); here that difference is an ``Engine`` and the loop is shared
(``engine/trainer.py``).
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class Engine:
    name = "base"
    model = None
    device: torch.device
    dp_group = None          # group over which batches differ (metrics are reduced here)
    dp_rank = 0
    dp_world = 1
    collective_generate = False  # True if generate must run on every rank
    is_logger = True          # this rank prints / saves
    scaler = None             # ops.amp.GradScaler when --grad_scaler (reference GradScaler)

    def _scaled(self, loss):
        return self.scaler.scale(loss) if self.scaler is not None else loss

    def _scaler_state(self) -> dict:
        return {"scaler": self.scaler.state_dict()} if self.scaler is not None else {}

    def _load_scaler_state(self, st: dict) -> None:
        if self.scaler is not None and st.get("scaler") is not None:
            self.scaler.load_state_dict(st["scaler"])

    def train_step(self, batch: dict, targets: torch.Tensor) -> torch.Tensor:
        """One optimizer step; returns the (local) mean loss as a 0-dim device tensor,
        or None on ranks that do not see the loss (non-last pipeline stages)."""
        raise NotImplementedError

    @torch.no_grad()
    def eval_step(self, batch: dict, targets: torch.Tensor):
        """Returns (loss_sum, n_valid, n_correct) device tensors (or None off the last stage)."""
        raise NotImplementedError

    def lm(self):
        """Callable(input_ids=, position_ids=) -> logits for ``generate``."""
        raise NotImplementedError

    def full_state_dict(self):
        """Canonical model state on the logging rank (collective for sharded engines)."""
        raise NotImplementedError

    def train_state(self) -> dict:
        raise NotImplementedError

    def load_train_state(self, st: dict) -> None:
        raise NotImplementedError

    def load_model_state(self, sd: dict) -> None:
        raise NotImplementedError

    @property
    def step_count(self) -> int:
        return 0

    def reset_step_state(self) -> None:
        """Forget the per-step bookkeeping of the store / pipeline -- collectives 'launched',
        gathered units, in-flight sends -- after a failed HIP-graph capture: nothing the
        capture recorded ever ran, so the eager retry must issue everything again (a bucket
        left marked as launched would never be all-reduced: silent rank divergence)."""
        from ..parallel import transport

        for obj in (getattr(self, "store", None), getattr(self, "p2p", None)):
            if obj is not None and hasattr(obj, "reset_step_state"):
                obj.reset_step_state()
        transport.forget_outstanding()  # --stream_check: the recorded handles never ran
        transport.reset_cu_reserve()


class GraphedStep:
    """The whole training step of an engine -- memset of the gradients, forward, backward with
    its collectives, optimizer -- captured once into ONE HIP graph and replayed: the
    cookbook's meaning of the reference's ``torch.compile`` (``/root/reference/main-ddp.py:60-61``,
    ``main-fsdp.py:74-75``, ``main-pipe.py:108-109``), without Inductor / Triton.

    Call 1 for an input signature runs eagerly (lazy init, allocator and communicator
    warm-up); call 2 captures the step against static input buffers and replays it; later
    calls copy the batch into the static buffers and replay.  The optimizers read their step
    count from a device counter (``FlatAdamW.device_step``), so a replay applies the right
    bias corrections.  Collectives must be capturable (native RCCL transport, or none at one
    rank).  If capture fails the engine stays eager and says so."""

    def __init__(self, engine, optimizers):
        self.engine = engine
        self.opts = list(optimizers)
        self.enabled = True
        self.graph = None
        self.key = None
        self.static = None
        self.loss = None

    # test seams: how a graph is made and captured (the CPU tests substitute a capture that
    # fails part-way through the step body)
    @staticmethod
    def _new_graph():
        return torch.cuda.CUDAGraph()

    @staticmethod
    def _capture(g, mode):
        return torch.cuda.graph(g, capture_error_mode=mode)

    def _sync(self):
        if self.engine.device.type == "cuda":
            torch.cuda.synchronize()

    @staticmethod
    def _watchdog():
        from ..parallel import native_comm

        return native_comm

    def __call__(self, body, batch, targets):
        if not self.enabled:
            return body(batch, targets)
        mask = batch.get("mask")
        key = (tuple(batch["input_ids"].shape), mask is None)
        if self.graph is not None and key == self.key:
            st = self.static
            st["ids"].copy_(batch["input_ids"], non_blocking=True)
            st["pos"].copy_(batch["position_ids"], non_blocking=True)
            st["tg"].copy_(targets, non_blocking=True)
            if mask is not None:
                st["mask"].copy_(mask, non_blocking=True)
            self._replay()
            for o in self.opts:
                o.step_count += 1
            return None if self.loss is None else self.loss.clone()
        if self.key != key:  # first call for this signature: eager (warm-up)
            self.key = key
            self.graph = None
            return body(batch, targets)
        st = {"ids": batch["input_ids"].clone(), "pos": batch["position_ids"].clone(),
              "tg": targets.clone(), "mask": None if mask is None else mask.clone()}
        self.static = st
        counts = [(o.step_count, o.device_step) for o in self.opts]
        for o in self.opts:
            o.device_step = True
        g = self._new_graph()
        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self._sync()
        if multi:
            # nothing of the process group may still be in flight when the capture starts
            dist.barrier()
            self._sync()
        wd = self._watchdog()
        native_wd = wd.watchdog_running()
        err = None
        try:
            # thread_local: only this thread's calls are checked -- the process group's and
            # the native watchdog threads keep querying their events while the capture runs
            # (the native one is also paused: no HIP call from it until the capture ends)
            wd.watchdog_pause(True)
            with self._capture(g, "thread_local" if (multi or native_wd) else "global"):
                b = {"input_ids": st["ids"], "position_ids": st["pos"], "mask": st["mask"]}
                self.loss = body(b, st["tg"])
        except Exception as exc:  # capture not possible: stay eager
            err = exc
        finally:
            wd.watchdog_pause(False)
        if multi:
            # every rank graphs or none does: a rank replaying while another runs eagerly
            # would still issue the same collectives, but a failed capture may have left
            # RCCL work half-recorded on one side only
            flag = torch.tensor([0.0 if err is None else 1.0], device=self.engine.device)
            dist.all_reduce(flag)
            if err is None and float(flag.item()) > 0:
                err = RuntimeError("capture failed on another rank")
        if err is not None:
            # the capture recorded work that never ran: undo its host-side effects (optimizer
            # step counts, collectives marked as launched, gathered units) before the step is
            # run eagerly
            for o, (n, ds) in zip(self.opts, counts):
                o.step_count, o.device_step = n, ds
            self.engine.reset_step_state()
            self.enabled = False
            self.graph = None
            self.loss = None
            if self.engine.is_logger:
                print(f"[hip-graph] capture failed ({err!r}); running eagerly")
            self._sync()
            return body(batch, targets)
        self.graph = g
        self._replay()  # (the first replay right after the capture is watched too)
        return None if self.loss is None else self.loss.clone()

    def _replay(self):
        """Replay the step graph; the collectives inside it are watched as one unit by the
        native watchdog (its event is recorded behind the replay)."""
        self.graph.replay()
        wd = self._watchdog()
        if wd.watchdog_running():
            wd.watchdog_track(torch.cuda.current_stream().cuda_stream, "hip-graph step replay")
