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
* ``split`` builds sub-communicators (the PP x DP mesh) with ``ncclCommSplit``;
* a native watchdog thread (``rccl_comm.cpp``, ``dpc_wd_*``) follows every collective the
  transport enqueues with an event, polls those events and ``ncclCommGetAsyncError``, and on
  a collective pending past ``DPC_COLL_TIMEOUT`` seconds (default 1800, the c10d default the
  reference relied on) or an RCCL error calls ``ncclCommAbort`` on every communicator and
  exits the process non-zero (``DPC_WATCHDOG_EXIT``, default 17) -- torchrun then tears the
  job down (reference: c10d's watchdog + ``destroy_process_group``,
  ``/root/reference/main-ddp.py:26,34-35``);
* bring-up is agreed across the group: a rank that cannot load RCCL or draw the unique id
  still joins the id broadcast (with an error marker) and every rank raises together, so the
  caller's fallback to torch.distributed is taken by all ranks or none.

Every engine uses this communicator at N > 1 on a GPU by default (``parallel/transport.py``,
``--comm auto``); ``--comm torch`` selects torch's ``nccl`` process group (RCCL as well).
``DPC_RCCL_LIB`` / ``DPC_HIP_LIB`` force other RCCL / HIP libraries (the CPU tests' fakes).
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
            "dpc_rccl_load": ([ctypes.c_char_p, I], I),
            "dpc_hip_load": ([ctypes.c_char_p, I], I),
            "dpc_rccl_abort": ([P], I),
            "dpc_wd_start": ([ctypes.c_double, I, I, I], I),
            "dpc_wd_running": ([], I),
            "dpc_wd_register": ([P], None),
            "dpc_wd_unregister": ([P], None),
            "dpc_wd_track": ([P, ctypes.c_char_p], I),
            "dpc_wd_pending": ([], I),
            "dpc_wd_pause": ([I], None),
            "dpc_wd_stop": ([], None),
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
        tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
        forced = os.environ.get("DPC_RCCL_LIB")
        if h.dpc_rccl_load((forced or os.path.join(tlib, "librccl.so")).encode(), 1 if forced else 0) != 0:
            raise RuntimeError(f"native RCCL unavailable: {h.dpc_rccl_error().decode()}")
        _bound = h
    return _bound


# ---------------------------------------------------------------- watchdog (rccl_comm.cpp)
def watchdog_start(rank: int = 0) -> bool:
    """Start the native collective watchdog once per process (``DPC_WATCHDOG=0`` disables).
    Returns whether it runs."""
    if os.environ.get("DPC_WATCHDOG", "1") == "0":
        return False
    h = _lib()
    if h.dpc_wd_running():
        return True
    forced = os.environ.get("DPC_HIP_LIB")
    hip = forced or os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if h.dpc_hip_load(hip.encode(), 1 if forced else 0) != 0:
        return False
    timeout = float(os.environ.get("DPC_COLL_TIMEOUT", "1800"))
    poll_ms = int(os.environ.get("DPC_WATCHDOG_POLL_MS", "200"))
    code = int(os.environ.get("DPC_WATCHDOG_EXIT", "17"))
    return h.dpc_wd_start(timeout, poll_ms, rank, code) == 0


def watchdog_running() -> bool:
    return _bound is not None and bool(_bound.dpc_wd_running())


def watchdog_track(stream_ptr: int, desc: str) -> None:
    """Watch the work just enqueued on ``stream_ptr`` (no-op while not running)."""
    if _bound is not None and _bound.dpc_wd_running():
        _bound.dpc_wd_track(ctypes.c_void_p(stream_ptr), desc.encode())


def watchdog_pause(on: bool) -> None:
    """Pause the watchdog's HIP calls (around a HIP-graph capture)."""
    if _bound is not None:
        _bound.dpc_wd_pause(1 if on else 0)


def watchdog_pending() -> int:
    return int(_bound.dpc_wd_pending()) if _bound is not None else 0


def watchdog_stop() -> None:
    if _bound is not None:
        _bound.dpc_wd_stop()


def _agree(ok: bool, group) -> bool:
    """Whether every rank of ``group`` reports ``ok`` (one MIN all-reduce over the bootstrap
    process group; a 1-rank group trivially agrees)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return ok
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


_ERR = b"DPC-ERR:"


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
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        if device is not None and torch.device(device).type == "cuda":
            torch.cuda.set_device(device)
        # 1. library + unique id; rank 0 broadcasts the id or an error marker, so no peer is
        #    left waiting in the broadcast when rank 0 cannot build one
        err = None
        lib = None
        try:
            lib = _lib()
        except Exception as exc:  # noqa: BLE001 -- reported through the agreement below
            err = str(exc)
        payload = b""
        if self.rank == 0:
            uid = ctypes.create_string_buffer(128)
            if lib is not None and lib.dpc_rccl_unique_id(uid) == 0:
                payload = bytes(uid.raw)
            else:
                err = err or f"ncclGetUniqueId: {lib.dpc_rccl_error().decode() if lib else '?'}"
                payload = _ERR + err.encode()[:100]
        obj = [payload]
        src = dist.get_global_rank(group, 0) if group is not None else 0
        dist.broadcast_object_list(obj, src=src, group=group)
        if obj[0].startswith(_ERR):
            err = err or "rank 0: " + obj[0][len(_ERR):].decode(errors="replace")
        # 2. every rank enters ncclCommInitRank (itself collective) or none does
        if not _agree(err is None, group):
            raise RuntimeError(f"native RCCL bring-up refused ({err or 'failed on another rank'})")
        handle = ctypes.c_void_p()
        rc = lib.dpc_rccl_init(obj[0], self.size, self.rank, ctypes.byref(handle))
        ok = rc == 0
        if not _agree(ok, group):
            if ok and handle:
                lib.dpc_rccl_destroy(handle)
            raise RuntimeError(f"ncclCommInitRank failed ({lib.dpc_rccl_error().decode() if not ok else 'on another rank'})")
        self.comm = handle
        if watchdog_start(dist.get_rank()):
            lib.dpc_wd_register(self.comm)

    # ---------------------------------------------------------------- helpers
    @staticmethod
    def _stream(stream) -> int:
        if isinstance(stream, int):
            return stream
        if stream is None and not torch.cuda.is_available():
            return 0  # host-side fake library (CPU tests)
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
        """Sub-communicator of the ranks sharing ``color`` (ordered by ``key``), collective.

        ncclCommSplit is itself a blocking collective on this communicator, so the ranks first
        agree (through the bootstrap group) that every one of them can enter it: the parent is
        alive and reports no asynchronous error.  A rank that fails INSIDE the split after that
        leaves the others blocked in it; the native watchdog (``dpc_wd_*``) is what ends such a
        hang (abort + non-zero exit).  A split that returns an error on some rank is agreed
        afterwards: every rank keeps its split, or none does."""
        pre_ok = bool(self.comm) and _lib().dpc_rccl_async_error(self.comm) == 0
        if not _agree(pre_ok, self.group):
            raise RuntimeError("ncclCommSplit not attempted: the parent communicator is down on "
                               + ("this rank" if not pre_ok else "another rank"))
        out = ctypes.c_void_p()
        rc = _lib().dpc_rccl_split(self.comm, color, key, ctypes.byref(out))
        if not _agree(rc == 0, self.group):  # every rank keeps its split, or none does
            if rc == 0 and out:
                _lib().dpc_rccl_destroy(out)
            raise RuntimeError(f"ncclCommSplit failed ({_lib().dpc_rccl_error().decode() if rc else 'on another rank'})")
        # size/rank of the new communicator: count colours through the bootstrap group
        colors = [None] * self.size
        dist.all_gather_object(colors, (color, key, self.rank), group=self.group)
        members = sorted((k, r) for c, k, r in colors if c == color)
        rank = [r for _, r in members].index(self.rank)
        if watchdog_running():
            _lib().dpc_wd_register(out)
        return NativeComm(self.group, _handle=out, _rank=rank, _size=len(members))

    def check_async(self) -> None:
        _check(_lib().dpc_rccl_async_error(self.comm), "async error")

    def destroy(self) -> None:
        if self.comm:
            _lib().dpc_wd_unregister(self.comm)
            _check(_lib().dpc_rccl_destroy(self.comm), "ncclCommDestroy")
            self.comm = None

    def abort(self) -> None:
        """ncclCommAbort: tear the communicator down without waiting for peers."""
        if self.comm:
            _lib().dpc_wd_unregister(self.comm)
            _lib().dpc_rccl_abort(self.comm)
            self.comm = None
