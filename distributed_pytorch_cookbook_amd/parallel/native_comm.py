"""Native RCCL communicator (``runtime/csrc/rccl_comm.cpp``) for the engines' hot-path collectives.

SURVEY.md §2.4/§5.8 target: a C++ communicator over RCCL with explicit HIP streams, using
torch's process group only for bootstrap.  This class is that communicator:

* bootstrap: rank 0 of the group draws an ``ncclUniqueId`` and it is broadcast with
  ``torch.distributed.broadcast_object_list`` over the existing (TCPStore-rendezvoused)
  process group -- the reference's ``init_process_group("nccl")`` rendezvous
  (``/root/reference/main-ddp.py:26``) -- then every rank calls ``ncclCommInitRank``;
* collectives are enqueued on the caller's current torch stream (or an explicit one) with
  no c10d work objects: all-reduce (DDP buckets), reduce-scatter / all-gather (FSDP
  shards), broadcast (initial weights), grouped send/recv (pipeline activations);
* ``split`` builds sub-communicators (the PP x DP mesh) with ``ncclCommSplit``.

The engines use it when ``DPC_COMM=native`` (``--comm native``); the default remains
torch's ``nccl`` process group, which is RCCL as well.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch
import torch.distributed as dist

_DTYPES = {torch.int8: 0, torch.uint8: 1, torch.int32: 2, torch.int64: 4, torch.float16: 6,
           torch.float32: 7, torch.float64: 8, torch.bfloat16: 9}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}

_bound = None


def _lib():
    """The runtime library with the dpc_rccl_* entry points bound and RCCL resolved."""
    global _bound
    if _bound is None:
        from ..runtime import lib as runtime_lib

        h = runtime_lib()
        P, I, S = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
        sig = {
            "dpc_rccl_load": ([ctypes.c_char_p], I),
            "dpc_rccl_error": ([], ctypes.c_char_p),
            "dpc_rccl_unique_id": ([ctypes.c_char_p], I),
            "dpc_rccl_init": ([ctypes.c_char_p, I, I, ctypes.POINTER(P)], I),
            "dpc_rccl_split": ([P, I, I, ctypes.POINTER(P)], I),
            "dpc_rccl_destroy": ([P], I),
            "dpc_rccl_async_error": ([P], I),
            "dpc_rccl_all_reduce": ([P, P, P, S, I, I, P], I),
            "dpc_rccl_reduce_scatter": ([P, P, P, S, I, I, P], I),
            "dpc_rccl_all_gather": ([P, P, P, S, I, P], I),
            "dpc_rccl_broadcast": ([P, P, P, S, I, I, P], I),
            "dpc_rccl_send": ([P, P, S, I, I, P], I),
            "dpc_rccl_recv": ([P, P, S, I, I, P], I),
            "dpc_rccl_group_start": ([], I),
            "dpc_rccl_group_end": ([], I),
        }
        for name, (args, res) in sig.items():
            fn = getattr(h, name)
            fn.argtypes, fn.restype = args, res
        torch_rccl = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if h.dpc_rccl_load(torch_rccl.encode()) != 0:
            raise RuntimeError(f"native RCCL unavailable: {h.dpc_rccl_error().decode()}")
        _bound = h
    return _bound


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {_lib().dpc_rccl_error().decode()}")


class NativeComm:
    """An RCCL communicator over the ranks of ``group`` (default: the world)."""

    def __init__(self, group=None, device: torch.device | None = None, _handle=None, _rank=None, _size=None):
        self.group = group
        if _handle is not None:
            self.comm, self.rank, self.size = _handle, _rank, _size
            return
        lib = _lib()
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        if device is not None:
            torch.cuda.set_device(device)
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            _check(lib.dpc_rccl_unique_id(uid), "ncclGetUniqueId")
        obj = [bytes(uid.raw)]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        handle = ctypes.c_void_p()
        _check(lib.dpc_rccl_init(obj[0], self.size, self.rank, ctypes.byref(handle)), "ncclCommInitRank")
        self.comm = handle

    # ---------------------------------------------------------------- helpers
    @staticmethod
    def _stream(stream) -> int:
        s = stream if stream is not None else torch.cuda.current_stream()
        return s.cuda_stream

    @staticmethod
    def _dt(t: torch.Tensor) -> int:
        if t.dtype not in _DTYPES:
            raise TypeError(f"unsupported dtype {t.dtype}")
        if not t.is_contiguous():
            raise ValueError("RCCL buffers must be contiguous")
        return _DTYPES[t.dtype]

    # ---------------------------------------------------------------- collectives
    def all_reduce(self, t: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        _check(_lib().dpc_rccl_all_reduce(self.comm, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t),
                                          _OPS[op], self._stream(stream)), "all_reduce")
        return t

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", stream=None) -> torch.Tensor:
        if inp.numel() != out.numel() * self.size:
            raise ValueError("reduce_scatter: input must hold world_size x output elements")
        _check(_lib().dpc_rccl_reduce_scatter(self.comm, inp.data_ptr(), out.data_ptr(), out.numel(),
                                              self._dt(out), _OPS[op], self._stream(stream)), "reduce_scatter")
        return out

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, stream=None) -> torch.Tensor:
        if out.numel() != inp.numel() * self.size:
            raise ValueError("all_gather: output must hold world_size x input elements")
        _check(_lib().dpc_rccl_all_gather(self.comm, inp.data_ptr(), out.data_ptr(), inp.numel(),
                                          self._dt(inp), self._stream(stream)), "all_gather")
        return out

    def broadcast(self, t: torch.Tensor, src: int = 0, stream=None) -> torch.Tensor:
        _check(_lib().dpc_rccl_broadcast(self.comm, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), src,
                                         self._stream(stream)), "broadcast")
        return t

    def send(self, t: torch.Tensor, peer: int, stream=None) -> None:
        _check(_lib().dpc_rccl_send(self.comm, t.data_ptr(), t.numel(), self._dt(t), peer,
                                    self._stream(stream)), "send")

    def recv(self, t: torch.Tensor, peer: int, stream=None) -> torch.Tensor:
        _check(_lib().dpc_rccl_recv(self.comm, t.data_ptr(), t.numel(), self._dt(t), peer,
                                    self._stream(stream)), "recv")
        return t

    @contextlib.contextmanager
    def grouped(self):
        """Fuse the enclosed send/recv calls (ncclGroupStart / ncclGroupEnd)."""
        _check(_lib().dpc_rccl_group_start(), "group_start")
        try:
            yield self
        finally:
            _check(_lib().dpc_rccl_group_end(), "group_end")

    def split(self, color: int, key: int) -> "NativeComm":
        """Sub-communicator of the ranks sharing ``color`` (ordered by ``key``), collective."""
        out = ctypes.c_void_p()
        _check(_lib().dpc_rccl_split(self.comm, color, key, ctypes.byref(out)), "ncclCommSplit")
        # size/rank of the new communicator: count colours through the bootstrap group
        colors = [None] * self.size
        dist.all_gather_object(colors, (color, key, self.rank), group=self.group)
        members = sorted((k, r) for c, k, r in colors if c == color)
        rank = [r for _, r in members].index(self.rank)
        return NativeComm(self.group, _handle=out, _rank=rank, _size=len(members))

    def check_async(self) -> None:
        _check(_lib().dpc_rccl_async_error(self.comm), "async error")

    def destroy(self) -> None:
        if self.comm:
            _check(_lib().dpc_rccl_destroy(self.comm), "ncclCommDestroy")
            self.comm = None
