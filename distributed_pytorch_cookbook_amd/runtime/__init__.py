"""Native host runtime (C++): token-file batch loader, synthetic corpus generator, host AdamW.

See ``runtime/csrc/runtime.cpp``.  Loaded with ctypes; built in-tree by ``runtime/build.py``
(also from ``__graft_entry__.build``).
"""
from __future__ import annotations

import ctypes
import math
import threading
from ctypes import c_char_p, c_float, c_int, c_int64, c_uint64, c_void_p

import numpy as np
import torch

from . import build as _build

_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if _build.needs_build():
                    _build.build()
                h = ctypes.CDLL(str(_build.LIB_PATH))
                h.dpc_tokfile_open.argtypes = [c_char_p, c_int]
                h.dpc_tokfile_open.restype = c_void_p
                h.dpc_tokfile_len.argtypes = [c_void_p]
                h.dpc_tokfile_len.restype = c_int64
                h.dpc_tokfile_close.argtypes = [c_void_p]
                h.dpc_loader_create.argtypes = [c_void_p, c_int, c_int, c_uint64, c_int, c_int, c_int, c_int]
                h.dpc_loader_create.restype = c_void_p
                h.dpc_loader_next.argtypes = [c_void_p, c_void_p]
                h.dpc_loader_next.restype = c_int64
                h.dpc_loader_destroy.argtypes = [c_void_p]
                h.dpc_loader_seek.argtypes = [c_void_p, c_int64]
                h.dpc_synth_markov.argtypes = [c_void_p, c_int64, c_int, c_int, c_uint64, c_int, c_int64]
                h.dpc_adamw_host.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int64] + [c_float] * 8 + [c_void_p]
                _lib = h
    return _lib


def synth_markov(rows: int, seq_len: int, vocab: int = 50257, seed: int = 0, branching: int = 4,
                 row0: int = 0) -> torch.Tensor:
    out = torch.empty(rows, seq_len, dtype=torch.int64)
    lib().dpc_synth_markov(out.data_ptr(), rows, seq_len, vocab, seed, branching, row0)
    return out


def adamw_host(p, g, m, v, lr, b1, b2, eps, wd, step, grad_scale=1.0, shadow=None):
    """Fused host AdamW over flat f32 CPU tensors (+ optional bf16 host copy)."""
    for t in (p, g, m, v):
        assert t.device.type == "cpu" and t.dtype == torch.float32 and t.is_contiguous()
    bc1 = 1.0 - b1 ** step
    bc2s = math.sqrt(1.0 - b2 ** step)
    sh = None
    if shadow is not None:
        assert shadow.dtype == torch.bfloat16 and shadow.device.type == "cpu"
        sh = shadow.data_ptr()
    lib().dpc_adamw_host(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(), lr, b1, b2,
                         eps, wd, bc1, bc2s, grad_scale, sh)


class TokenFile:
    """Memory-mapped flat token file (uint16 or uint32 ids)."""

    def __init__(self, path: str, width: int = 2):
        self.h = lib().dpc_tokfile_open(str(path).encode(), width)
        if not self.h:
            raise FileNotFoundError(f"cannot map token file {path}")
        self.path, self.width = path, width

    def __len__(self):
        return int(lib().dpc_tokfile_len(self.h))

    def close(self):
        if self.h:
            lib().dpc_tokfile_close(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class NativeBatchLoader:
    """Infinite iterator of ``{"input_ids": [B, S+1], "attention_mask": ones}`` batches cut from
    a token file by native worker threads (deterministic, disjoint per DP rank)."""

    def __init__(self, tokfile: TokenFile, batch_size: int, seq_len: int, seed: int = 0, rank: int = 0,
                 world: int = 1, threads: int = 4, depth: int = 8):
        self.tf = tokfile
        self.B, self.S = batch_size, seq_len - 1  # windows of seq_len tokens
        self.h = lib().dpc_loader_create(tokfile.h, self.B, self.S, seed, rank, world, threads, depth)
        if not self.h:
            raise RuntimeError("loader creation failed")
        self.buf = torch.empty(self.B, self.S + 1, dtype=torch.int64,
                               pin_memory=torch.cuda.is_available())

    def __iter__(self):
        return self

    def __next__(self):
        lib().dpc_loader_next(self.h, self.buf.data_ptr())
        ids = self.buf.clone()
        return {"input_ids": ids, "attention_mask": torch.ones_like(ids)}

    def seek(self, batch_index: int) -> None:
        """Continue the stream at ``batch_index`` (nothing before it is loaded)."""
        lib().dpc_loader_seek(self.h, int(batch_index))

    def close(self):
        if self.h:
            lib().dpc_loader_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def write_token_file(path: str, tokens, width: int = 2) -> None:
    arr = np.asarray(tokens, dtype=np.uint16 if width == 2 else np.uint32)
    arr.tofile(path)
