"""Fused AdamW over flat buffers.

Reference: ``torch.optim.AdamW(model.parameters(), lr=args.learning_rate)``
(``/root/reference/main-single.py:42``; defaults betas=(0.9, 0.999), eps=1e-8,
weight_decay=1e-2, decoupled decay applied to every parameter).  Here the whole model
(or the local FSDP shard) is ONE contiguous f32 buffer, so a step is one kernel launch
that also refreshes the bf16 compute copy of the weights.
"""
from __future__ import annotations

import math

import torch

from . import _lib


class FlatAdamW:
    def __init__(self, param: torch.Tensor, grad: torch.Tensor, lr: float = 1e-3,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 shadow: torch.Tensor | None = None):
        assert param.dim() == 1 and param.shape == grad.shape and param.dtype == torch.float32
        self.param, self.grad, self.shadow = param, grad, shadow
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.exp_avg = torch.zeros_like(param)
        self.exp_avg_sq = torch.zeros_like(param)
        self.step_count = 0
        # device-side step counter: lets a captured HIP graph replay the update with the
        # right bias corrections every step (host scalars would be frozen at capture)
        self.step_t = torch.zeros((), device=param.device, dtype=torch.float32)
        self.device_step = False

    def state_dict(self):
        return {"step": self.step_count, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "lr": self.lr, "betas": self.betas, "eps": self.eps,
                "weight_decay": self.weight_decay}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])

    @torch.no_grad()
    def step(self, grad_scale: float = 1.0, grad_scale_t: torch.Tensor | None = None,
             skip_t: torch.Tensor | None = None) -> None:
        self.begin_step(skip_t)
        self.update(0, self.param.numel(), grad_scale, grad_scale_t, skip_t)

    def begin_step(self, skip_t: torch.Tensor | None = None) -> None:
        """Advance the step count (host and, for HIP-graph replay, device counter).  With a
        loss scaler, ``skip_t`` (device flag) keeps a skipped step out of the device count
        that the bias corrections read (torch's GradScaler skips ``optimizer.step``)."""
        self.step_count += 1
        p = self.param
        if p.is_cuda and p.numel() % 4 == 0:
            if skip_t is not None:
                self.device_step = True
                self.step_t.add_(1.0).sub_(skip_t.to(self.step_t.dtype))
            elif self.device_step:
                self.step_t.add_(1.0)
            else:
                self.step_t.fill_(float(self.step_count))
        elif skip_t is not None:
            self.step_t.add_(1.0).sub_(skip_t.to(self.step_t.device, self.step_t.dtype))

    @torch.no_grad()
    def update(self, lo: int, hi: int, grad_scale: float = 1.0,
               grad_scale_t: torch.Tensor | None = None, skip_t: torch.Tensor | None = None) -> None:
        """Apply the current step to elements [lo, hi) of the flat buffers -- lets DDP update
        the buckets whose all-reduce has finished while the last one is still on the links."""
        b1, b2 = self.betas
        bc1 = 1.0 - b1 ** self.step_count
        bc2s = math.sqrt(1.0 - b2 ** self.step_count)
        p, g = self.param, self.grad
        if p.is_cuda and p.numel() % 4 == 0 and lo % 4 == 0 and (hi - lo) % 4 == 0:
            if hi <= lo:
                return
            f4 = 4 * lo
            args = _lib.AdamArgs(
                param=p.data_ptr() + f4, grad=g.data_ptr() + f4, exp_avg=self.exp_avg.data_ptr() + f4,
                exp_avg_sq=self.exp_avg_sq.data_ptr() + f4,
                shadow=(self.shadow.data_ptr() + lo * self.shadow.element_size()) if self.shadow is not None else None,
                grad_scale_ptr=_lib.ptr(grad_scale_t), n=hi - lo, lr=self.lr, beta1=b1,
                beta2=b2, eps=self.eps, weight_decay=self.weight_decay, bias_correction1=bc1,
                bias_correction2_sqrt=bc2s, grad_scale=grad_scale,
                step_ptr=self.step_t.data_ptr() if self.device_step else None,
                skip_ptr=_lib.ptr(skip_t),
            )
            _lib.call("dpc_adamw", args, p.device)
            return
        # (other paths: elements [lo, hi) through views -- FSDP updates unit shards one by one)
        p, g = p[lo:hi], g[lo:hi]
        m_, v_ = self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi]
        sh = None if self.shadow is None else self.shadow[lo:hi]
        if skip_t is not None:
            # non-HIP paths: a host-read flag (the CPU / offload paths synchronise anyway)
            if float(skip_t) != 0.0:
                return
            t = float(self.step_t)  # counted without the skipped steps
            bc1, bc2s = 1.0 - b1 ** t, math.sqrt(1.0 - b2 ** t)
        if p.device.type == "cpu" and grad_scale_t is not None and grad_scale_t.numel() == 1:
            grad_scale, grad_scale_t = grad_scale * float(grad_scale_t), None  # host path: a scalar
        if p.device.type == "cpu" and grad_scale_t is None and g.device.type == "cpu":
            # host path (FSDP --cpu_offload): one fused native pass (runtime/csrc/runtime.cpp)
            try:
                from .. import runtime

                host_shadow = None
                bf16_shadow = sh is not None and sh.dtype == torch.bfloat16
                if bf16_shadow:
                    if getattr(self, "_host_shadow", None) is None:
                        self._host_shadow = torch.empty(self.param.numel(), dtype=torch.bfloat16,
                                                        pin_memory=torch.cuda.is_available())
                    host_shadow = self._host_shadow[lo:hi]
                hstep = int(round(float(self.step_t))) if skip_t is not None else self.step_count
                runtime.adamw_host(p, g, m_, v_, self.lr, b1, b2, self.eps,
                                   self.weight_decay, hstep, grad_scale, host_shadow)
                if bf16_shadow:
                    sh.copy_(host_shadow, non_blocking=True)
                elif sh is not None:
                    sh.copy_(p, non_blocking=True)
                return
            except (ImportError, OSError, RuntimeError):
                pass
        gs = g * grad_scale
        if grad_scale_t is not None:
            gs = gs * grad_scale_t
        p.mul_(1.0 - self.lr * self.weight_decay)
        m_.mul_(b1).add_(gs, alpha=1 - b1)
        v_.mul_(b2).addcmul_(gs, gs, value=1 - b2)
        denom = (v_.sqrt() / bc2s).add_(self.eps)
        p.addcdiv_(m_, denom, value=-self.lr / bc1)
        if sh is not None:
            sh.copy_(p)
