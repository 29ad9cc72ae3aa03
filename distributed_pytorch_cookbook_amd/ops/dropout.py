"""Counter-based dropout (reference ``nn.Dropout`` sites, ``/root/reference/models/gpt.py:31,40,65,103``).

The reference applies dropout to the FFN output (after the second activation) and to the
attention output projection, each right before its residual add.  Here the keep mask of
a ``[T, N]`` site is a pure function of ``(key, t * N + c)``::

    keep(t, c) = fmix32(((t * N + c) * 0x9E3779B1) mod 2^32  xor  key) >= thresh

(``fmix32`` = MurmurHash3's finaliser), with ``key`` derived from a per-step seed and the
site number, and ``thresh = round(p * 2^32)``.  Nothing is saved for the backward: the
backward kernel regenerates the same mask.  Because the map is a bijection of the element
index for a fixed key, exactly ``p`` of the hash range is dropped.

``keep_mask`` is the bit-identical torch twin of the device hash (``misc.hip:fmix32``),
used by the CPU path and by the tests.
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from . import _lib

M32 = 0xFFFFFFFF


def _fmix32_int(x: int) -> int:
    x &= M32
    x ^= x >> 16
    x = (x * 0x85EBCA6B) & M32
    x ^= x >> 13
    x = (x * 0xC2B2AE35) & M32
    x ^= x >> 16
    return x


def _fmix32_t(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & M32
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & M32
    return x ^ (x >> 16)


@dataclass(frozen=True, eq=False)
class DropSpec:
    """Dropout of one site for one forward: keep iff hash >= thresh, kept values * scale.

    ``seed_t`` (optional): the forward's seed in device memory, int32 [2] = (low word, high
    word).  The kernels then derive the key from it themselves (``common.h:drop_key_of``, the
    same hash as ``key``), so a HIP-graph replay of the step draws fresh masks each step: the
    model advances the device counter with a captured add (``gpt.py:next_dropout_seed``)."""

    key: int
    thresh: int
    scale: float
    seed_t: "torch.Tensor | None" = None
    site: int = 0

    @staticmethod
    def make(p: float, seed: int, site: int, seed_t: "torch.Tensor | None" = None) -> "DropSpec | None":
        if p <= 0.0:
            return None
        if p >= 1.0:
            raise ValueError("dropout probability must be < 1")
        key = _fmix32_int(_fmix32_int(seed & M32) ^ _fmix32_int((seed >> 32) + 0x632BE5AB * (site + 1)))
        thresh = min(int(round(p * 2.0 ** 32)), M32)
        return DropSpec(key, thresh, 1.0 / (1.0 - p), seed_t, site)

    def seed_ptr(self):
        return self.seed_t.data_ptr() if self.seed_t is not None and self.seed_t.is_cuda else None


def keep_mask(spec: DropSpec, T: int, N: int, device=None) -> torch.Tensor:
    """f32 [T, N] tensor of 0 / scale, bit-identical to the device kernels' mask."""
    idx = torch.arange(T * N, device=device, dtype=torch.int64)
    h = _fmix32_t(((idx * 0x9E3779B1) & M32) ^ spec.key)
    return (h >= spec.thresh).to(torch.float32).mul_(spec.scale).reshape(T, N)


def dropout_residual(y: torch.Tensor, res: torch.Tensor, spec: DropSpec,
                     out: torch.Tensor | None = None) -> torch.Tensor:
    """``out = res + y * keep / (1 - p)`` on f32 [T, N] (``out`` may alias ``y`` or ``res``)."""
    T, N = y.shape
    if out is None:
        out = torch.empty_like(res)
    if not y.is_cuda:
        out.copy_(res + y * keep_mask(spec, T, N, y.device))
        return out
    for t in (y, res, out):
        if t.dtype != torch.float32 or t.stride(1) != 1 or t.stride(0) % 4:
            raise ValueError("dropout_residual: f32 operands with contiguous, 16-B aligned rows")
    if N % 4 or T * N >= 2 ** 32:
        raise ValueError("dropout_residual: N % 4 == 0 and T * N < 2^32 required")
    args = _lib.DropResArgs(
        y=y.data_ptr(), res=res.data_ptr(), out=out.data_ptr(),
        ldy=y.stride(0), ldr=res.stride(0), ldo=out.stride(0), T=T, N=N,
        key=spec.key, thresh=spec.thresh, scale=spec.scale, seed=spec.seed_ptr(), site=spec.site,
    )
    _lib.call("dpc_dropout_residual", args, y.device)
    return out
