"""Dynamic loss scaling -- the reference's ``torch.cuda.amp.GradScaler``, fused.

Reference: ``scaler = torch.cuda.amp.GradScaler()`` then ``scaler.scale(loss).backward();
scaler.step(optim); scaler.update()`` in every recipe (``/root/reference/main-single.py:78,
99-101``, ``main-ddp.py:122-126``, ``main-fsdp.py:136-140``).  torch's version launches a
multi-tensor unscale + non-finite check over every gradient tensor, a host-side skip
decision and an update kernel.  Here:

* ``scale(loss)`` multiplies the loss by the device scale, so the fused backward (whose
  head reads ``dloss`` as the GEMM alpha) produces scaled gradients;
* ``check(grad_flat)`` is ONE read of the flat gradient buffer (``amp_check_kernel``) that
  raises a device flag -- the 1/scale unscale is folded into the AdamW kernel
  (``grad_scale_ptr``), and the same flag makes AdamW leave parameters / moments untouched
  (``skip_ptr``) and keeps the skipped step out of the bias-correction count;
* ``update()`` is a one-thread kernel: back off on overflow, grow after ``growth_interval``
  clean steps (torch defaults: 2^16, x2, x0.5, 2000).

Nothing reads the flag on the host, so the whole step still replays as one HIP graph.
With bf16 compute the scaler is numerically unnecessary (the reference keeps it anyway);
``--grad_scaler`` enables it.  Sharded gradients (FSDP shards, pipeline stages) reduce the
flag over the process group so every rank takes the same decision.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib


class GradScaler:
    def __init__(self, device, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000):
        dev = torch.device(device)
        self.device = dev
        self.scale_t = torch.full((), init_scale, device=dev, dtype=torch.float32)
        self.inv_scale_t = torch.full((), 1.0 / init_scale, device=dev, dtype=torch.float32)
        self.found_inf = torch.zeros((), device=dev, dtype=torch.float32)
        self.tracker = torch.zeros((), device=dev, dtype=torch.float32)
        self.growth, self.backoff, self.interval = growth_factor, backoff_factor, int(growth_interval)

    # ------------------------------------------------------------------ step pieces
    def scale(self, loss: torch.Tensor) -> torch.Tensor:
        return loss * self.scale_t.to(loss.dtype)

    @torch.no_grad()
    def check(self, grad: torch.Tensor) -> None:
        """found_inf |= any non-finite element of ``grad`` (flat f32 buffer, any device)."""
        if grad.numel() == 0:
            return
        if grad.is_cuda and grad.dtype == torch.float32 and grad.is_contiguous() and self.found_inf.is_cuda:
            _lib.call("dpc_amp_check", _lib.AmpCheckArgs(g=grad.data_ptr(), n=grad.numel(),
                                                         found_inf=self.found_inf.data_ptr()), grad.device)
            return
        bad = (~torch.isfinite(grad)).any().to(self.found_inf.device, torch.float32)
        self.found_inf.copy_(torch.maximum(self.found_inf, bad))

    @torch.no_grad()
    def reduce_flag(self, group=None) -> None:
        """Every rank of ``group`` skips if any rank saw a non-finite gradient."""
        if dist.is_initialized() and dist.get_world_size(group) > 1:
            dist.all_reduce(self.found_inf, op=dist.ReduceOp.MAX, group=group)

    @torch.no_grad()
    def update(self) -> None:
        if self.scale_t.is_cuda:
            _lib.call("dpc_amp_update", _lib.AmpUpdateArgs(
                scale=self.scale_t.data_ptr(), inv_scale=self.inv_scale_t.data_ptr(),
                found_inf=self.found_inf.data_ptr(), tracker=self.tracker.data_ptr(),
                growth=self.growth, backoff=self.backoff, interval=self.interval), self.device)
            return
        inf = bool(self.found_inf.item())
        if inf:
            self.scale_t.mul_(self.backoff)
            self.tracker.zero_()
        else:
            self.tracker.add_(1.0)
            if self.tracker.item() >= self.interval:
                self.scale_t.mul_(self.growth)
                self.tracker.zero_()
        self.inv_scale_t.copy_(1.0 / self.scale_t)
        self.found_inf.zero_()

    def opt_kwargs(self, opt) -> dict:
        """``grad_scale_t`` / ``skip_t`` for ``FlatAdamW.step`` / ``update``, on the
        optimizer's device (a host-resident optimizer -- FSDP ``--cpu_offload`` -- gets host
        copies: that path synchronises anyway)."""
        dev = opt.param.device
        if dev == self.device:
            return {"grad_scale_t": self.inv_scale_t, "skip_t": self.found_inf}
        return {"grad_scale_t": self.inv_scale_t.to(dev), "skip_t": self.found_inf.to(dev)}

    # ------------------------------------------------------------------ state
    def state_dict(self) -> dict:
        return {"scale": float(self.scale_t), "growth_tracker": float(self.tracker)}

    def load_state_dict(self, sd: dict) -> None:
        self.scale_t.fill_(float(sd["scale"]))
        self.inv_scale_t.fill_(1.0 / float(sd["scale"]))
        self.tracker.fill_(float(sd.get("growth_tracker", 0.0)))
