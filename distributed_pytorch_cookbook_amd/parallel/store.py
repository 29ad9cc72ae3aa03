"""Parameter stores: flat f32 master weights + compute copies + f32 gradient buffers.

The reference keeps every parameter as its own tensor and lets torch's DDP Reducer / FSDP
FlatParameter repack them (``main-ddp.py:55``, ``main-fsdp.py:60-69``).  Here the model's
parameters are *views into one flat buffer* from the start, laid out unit by unit
(embeddings | layer 0 | ... | layer L-1 | head), each parameter 64-element aligned:

* the optimizer is one fused kernel over the flat buffer (``ops/optim.py``);
* DDP buckets are contiguous slices of the flat gradient buffer -- no copy in or out;
* FSDP shards are contiguous slices of a unit's range;
* the bf16 compute copy of every matrix is refreshed by the optimizer kernel itself, so
  the forward never casts weights;
* Q, K and V of a layer are adjacent, so the fused QKV GEMM uses a view.

Stores expose ``weight(p)`` (compute view: bf16 for matrices on a HIP device, the f32
master for vectors and on CPU), ``grad(p)`` (f32 view the kernels accumulate into) and
unit hooks (``pre/post_forward``, ``pre/post_backward``) that the fused model calls at
unit boundaries; parallel engines subclass and act in those hooks.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from ..ops.elementwise import cast_f32_bf16

ALIGN = 64  # elements


def _round(n: int, a: int) -> int:
    return (n + a - 1) // a * a


@dataclass
class Entry:
    name: str
    param: nn.Parameter
    unit: int
    offset: int  # absolute offset in the full flat layout
    numel: int
    shape: torch.Size


class FlatLayout:
    """Canonical flat layout of a model's parameters, unit by unit."""

    def __init__(self, model, unit_align: int = ALIGN):
        self.units = model.units()
        self.unit_names = [n for n, _ in self.units]
        self.entries: list[Entry] = []
        self.by_param: dict[int, Entry] = {}
        self.unit_ranges: list[tuple[int, int]] = []
        names = {id(p): n for n, p in model.named_parameters()}
        off = 0
        for ui, (_, mods) in enumerate(self.units):
            start = off
            for mod in mods:
                for p in mod.parameters():
                    e = Entry(names[id(p)], p, ui, off, p.numel(), p.shape)
                    self.entries.append(e)
                    self.by_param[id(p)] = e
                    # a matrix flagged ``_dpc_pad_rows`` (the lm_head) gets zero rows up to
                    # that multiple right after it, so a row-padded view (vocab 50257 ->
                    # 50304) is a plain [Vp, D] operand; the zeros stay zero (grad 0, decay 0)
                    reserve = p.numel()
                    pad = getattr(p, "_dpc_pad_rows", 0)
                    if pad and p.dim() == 2:
                        reserve = _round(p.shape[0], pad) * p.shape[1]
                    off += _round(reserve, ALIGN)
            end = _round(off, unit_align)
            self.unit_ranges.append((start, end))
            off = end
        self.total = off
        for ui, (_, mods) in enumerate(self.units):
            for mod in mods:
                object.__setattr__(mod, "_unit_id", ui)
        object.__setattr__(model, "_head_unit_id", len(self.units) - 1)

    def unit_entries(self, u: int):
        return [e for e in self.entries if e.unit == u]


def default_compute_dtype(device: torch.device) -> torch.dtype:
    return torch.bfloat16 if device.type == "cuda" else torch.float32


class ParamStore:
    """Interface used by ``models/fused.py``."""

    compute_dtype: torch.dtype
    anchor: torch.Tensor

    def weight(self, p):
        raise NotImplementedError

    def grad(self, p):
        raise NotImplementedError

    def pre_forward(self, u):
        pass

    def post_forward(self, u, training=True):
        pass

    def pre_backward(self, u, need_weights=True):
        pass

    def post_backward(self, u):
        pass


class LocalStore(ParamStore):
    """Whole model on one device (single-GPU recipe; base of the DDP store).

    ``units`` restricts the store to a subset of units (pipeline stages); parameters of
    other units are left untouched (typically on the meta device).
    """

    def __init__(self, model, device, compute_dtype=None, units=None, unit_align: int = ALIGN):
        device = torch.device(device)
        self.device = device
        self.compute_dtype = compute_dtype or default_compute_dtype(device)
        self.layout = FlatLayout(model, unit_align)
        self.units = list(range(len(self.layout.units))) if units is None else sorted(units)
        lo = self.layout.unit_ranges[self.units[0]][0]
        hi = self.layout.unit_ranges[self.units[-1]][1]
        assert all(self.layout.unit_ranges[a][1] == self.layout.unit_ranges[b][0]
                   for a, b in zip(self.units, self.units[1:])), "store units must be contiguous"
        self.base = lo
        self.numel = hi - lo
        self.master = torch.zeros(self.numel, device=device, dtype=torch.float32)
        self.grads = torch.zeros(self.numel, device=device, dtype=torch.float32)
        self.entries = [e for e in self.layout.entries if e.unit in set(self.units)]
        with torch.no_grad():
            for e in self.entries:
                view = self._view(self.master, e)
                src = e.param.data
                if src.device.type != "meta":
                    view.copy_(src)
                e.param.data = view
                e.param.grad = self._view(self.grads, e)
        self.shadow = None
        if self.compute_dtype != torch.float32:
            self.shadow = torch.empty(self.numel, device=device, dtype=self.compute_dtype)
            self.refresh_shadow()
        self.anchor = torch.zeros((), device=device, requires_grad=True)
        object.__setattr__(model, "param_store", self)
        self.model = model

    def _view(self, flat, e: Entry):
        o = e.offset - self.base
        return flat[o:o + e.numel].view(e.shape)

    def unit_slice(self, u: int) -> slice:
        a, b = self.layout.unit_ranges[u]
        return slice(a - self.base, b - self.base)

    def refresh_shadow(self):
        if self.shadow is not None:
            cast_f32_bf16(self.master, self.shadow)

    def weight(self, p):
        if self.shadow is not None and p.dim() >= 2:
            return self._view(self.shadow, self.layout.by_param[id(p)])
        return p.data

    def grad(self, p):
        return p.grad

    def zero_grad(self):
        self.grads.zero_()

    def named_entries(self):
        return [(e.name, e) for e in self.entries]

    def state_dict(self):
        """Canonical bare-key state dict of the units held here (views of the master)."""
        return {e.name: e.param.data for e in self.entries}

    def load_state_dict(self, sd, strict=True):
        missing = []
        with torch.no_grad():
            for e in self.entries:
                if e.name in sd:
                    e.param.data.copy_(sd[e.name])
                else:
                    missing.append(e.name)
        if strict and missing:
            raise KeyError(f"missing keys: {missing}")
        self.refresh_shadow()
