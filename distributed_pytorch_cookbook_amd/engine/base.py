"""Engine interface: what a recipe's training loop needs from a parallelism strategy.

The reference's recipes differ only in the wrapper around the model (SURVEY.md §1,
observation 2); here that difference is an ``Engine`` and the loop is shared
(``engine/trainer.py``).
"""
from __future__ import annotations

import torch


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
