"""One collective transport interface for every engine: native RCCL, torch c10d, or gloo.

SURVEY.md §2.4 / §5.8: the hot-path collectives of the three engines -- DDP bucket
all-reduces (reference ``/root/reference/main-ddp.py:55``), FSDP all-gathers and
reduce-scatters (``main-fsdp.py:60-69``) and pipeline send/recv (``main-pipe.py:75-83``) --
go through a ``Transport``:

* ``NativeTransport`` -- the C++ RCCL communicator (``runtime/csrc/rccl_comm.cpp`` via
  ``parallel/native_comm.py``).  Every collective is enqueued on the transport's own
  high-priority HIP stream, ordered after the caller's work by an event, and its completion
  is handed back as an event the caller's stream waits on (``Handle.wait``): no c10d work
  objects, no watchdog, no host synchronisation -- and therefore capturable in a HIP graph.
  Buffers touched on the comm stream are ``record_stream``-ed so the caching allocator does
  not recycle them while a collective still reads or writes them.
* ``TorchTransport`` -- torch.distributed over the same group: the ``nccl`` backend (RCCL
  as well) for ``--comm torch``, ``gloo`` for the CPU tests and shared-GPU rehearsals.

``make_transport`` picks native on a GPU with the nccl backend unless told otherwise, and
falls back to torch if the native library or RCCL cannot be brought up -- on every rank
together: ``NativeComm`` agrees each bring-up step over the bootstrap group
(``native_comm._agree``), so no rank is left inside a native collective while another has
moved on.  torch.distributed stays the bootstrap (rendezvous, the ``ncclUniqueId``
broadcast) and carries the few host-side scalar reductions.

Safety on the native path: ``--coll_check`` fingerprints every
native collective over the transport's torch group before it is enqueued (as
``TorchTransport`` does through ``comm.py``); every enqueued collective is watched by the
native watchdog (``native_comm.watchdog_*``: deadline + RCCL async errors -> ncclCommAbort
-> non-zero exit); ``shutdown_native`` -- called by ``comm.cleanup_dist`` -- destroys every
communicator and stops the watchdog.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from . import comm
from ..utils.profiling import mark


# ---------------------------------------------------------------- stream-order checks
# with DPC_STREAM_CHECK=1 (``--stream_check``) every asynchronous collective
# handle is registered when it is issued and struck off when a stream is ordered after it
# (``Handle.wait``); ``check_drained`` -- called by every engine at the end of its step --
# raises, naming the collectives, if any was never waited on (a consumer could have read its
# buffer before the collective finished), and polls each native communicator for an RCCL
# asynchronous error.  Buffers handed to the comm stream must be contiguous and on the
# transport's device; each is ``record_stream``-ed so the caching allocator cannot recycle
# it under the collective.
_STREAM_CHECK = os.environ.get("DPC_STREAM_CHECK", "0") == "1"
_outstanding: dict = {}
_native_comms: list = []


def set_stream_check(on: bool) -> None:
    global _STREAM_CHECK
    _STREAM_CHECK = bool(on)
    _outstanding.clear()


def stream_check_enabled() -> bool:
    return _STREAM_CHECK


def forget_outstanding() -> None:
    _outstanding.clear()


# ---------------------------------------------------------------- resident-CU reserve
# SURVEY.md §5.8 rule 4 (comm overlapped with compute on side streams): the persistent GEMMs
# (ops/csrc/gemm7.hip) size their grid to occupy every CU, so an RCCL kernel resident on a
# CU while a GEMM launches would push that CU's GEMM workgroup -- and its whole share of the
# tiles -- into a second round.  With DPC_CU_RESERVE=R, from the moment an asynchronous GPU
# collective is enqueued until its handle is waited on, the GEMMs leave R CUs free for it
# (captured into a HIP graph like every other launch parameter).  Default 0: on one MI355X the
# reserve itself costs a round of wave quantisation on the GPT-2 products (QKV forward +23 %,
# input gradient +40 % at R = 16 with nothing beside them) while a blocking collective-sized
# occupier costs a weight gradient +69 % -- and the handles are waited on only at the end of
# the backward, so a reserve would tax every backward GEMM (profiles/r3_gemm/cu_reserve*.log).
_CU_RESERVE = int(os.environ.get("DPC_CU_RESERVE", "0"))
_comm_inflight = 0


def _set_reserve(r: int) -> None:
    from ..ops import _lib

    try:
        _lib.set_cu_reserve(r)
    except (RuntimeError, OSError):  # no kernel library (CPU): nothing to size
        pass


def _reserve_begin() -> None:
    global _comm_inflight
    _comm_inflight += 1
    if _comm_inflight == 1 and _CU_RESERVE > 0:
        _set_reserve(_CU_RESERVE)


def _reserve_end() -> None:
    global _comm_inflight
    _comm_inflight = max(0, _comm_inflight - 1)
    if _comm_inflight == 0 and _CU_RESERVE > 0:
        _set_reserve(0)


def reset_cu_reserve() -> None:
    """No collective in flight (after a failed capture: the recorded ones never ran)."""
    global _comm_inflight
    if _comm_inflight:
        _comm_inflight = 0
        _set_reserve(0)


def cu_reserve_active() -> bool:
    return _comm_inflight > 0


# ---------------------------------------------------------------- fake collectives (one GPU)
# DPC_FAKE_COLL="<cus>,<bus GB/s>,<world>" (e.g. "16,300,8"): every collective of a native
# transport is followed, on its comm stream, by an occupier kernel of <cus> workgroups (32 KiB LDS
# each, so a CU hosting one cannot also host a persistent GEMM workgroup) that stays resident
# for the time the collective would take on <world> GPUs at <bus GB/s> bus bandwidth
# (all-reduce 2 (W-1) / W x bytes, reduce-scatter / all-gather (W-1) / W x the full buffer).
# Run at one rank (bench.py --force_dist_path), it reproduces the CU co-residency of the
# multi-GPU step -- the same launch points, sizes and overlap -- on a one-GPU box, to set
# DPC_CU_RESERVE from measurements (bench/cu_corun.sh).
# (parsed once at import; the occupier's sink is allocated when a NativeTransport is built --
# outside any HIP-graph capture, so a captured step never owns it)
_FAKE_COLL = tuple(float(v) for v in os.environ["DPC_FAKE_COLL"].split(",")) if os.environ.get("DPC_FAKE_COLL") else None
_fake_sink = None


def _fake_sink_for(device) -> None:
    global _fake_sink
    if _FAKE_COLL and _fake_sink is None and torch.device(device).type == "cuda":
        _fake_sink = torch.zeros(4096, dtype=torch.int32, device=device)


def _fake_coll(op: str, tensors, stream) -> None:
    from ..ops import _lib

    cus, busbw, world = _FAKE_COLL
    nbytes = max((t.numel() * t.element_size() for t in tensors), default=0)
    factor = {"all_reduce": 2.0 * (world - 1) / world, "reduce_scatter": (world - 1) / world,
              "all_gather": (world - 1) / world}.get(op, 1.0)
    ns = int(factor * nbytes / (busbw * 1e9) * 1e9)
    _lib.occupy(int(cus), ns, _fake_sink, stream)


def check_drained(where: str = "end of step") -> None:
    """Raise if a collective issued with ``async_op=True`` was never waited on."""
    if not _STREAM_CHECK:
        return
    for nc in _native_comms:
        nc.check_async()
    if _outstanding:
        pending = sorted(_outstanding.values())
        _outstanding.clear()
        raise RuntimeError(f"stream-order check: {len(pending)} collective(s) never waited on before "
                           f"{where}: {pending[:8]}")


class Handle:
    """Completion of an asynchronous collective."""

    def _track(self, desc: str) -> "Handle":
        if _STREAM_CHECK:
            _outstanding[id(self)] = desc
        return self

    def _untrack(self) -> None:
        if _outstanding:
            _outstanding.pop(id(self), None)

    def wait(self) -> None:  # pragma: no cover - interface
        raise NotImplementedError


class _Done(Handle):
    def wait(self) -> None:
        pass


class _EventHandle(Handle):
    """Completion recorded on a side stream: ``wait`` orders the caller's current stream
    after it (device-side only).  While it is outstanding the persistent GEMMs keep the
    resident-CU reserve (``_reserve_begin``)."""

    def __init__(self, event, reserved=False):
        self.event = event
        self.reserved = reserved

    def wait(self) -> None:
        self._untrack()
        torch.cuda.current_stream().wait_event(self.event)
        if self.reserved:
            self.reserved = False
            _reserve_end()


class _WorkHandle(Handle):
    def __init__(self, works, after=None):
        self.works = works if isinstance(works, (list, tuple)) else [works]
        self.after = after

    def wait(self) -> None:
        self._untrack()
        for w in self.works:
            if w is not None:
                w.wait()
        if self.after is not None:
            self.after()
            self.after = None


def _desc(op: str, tensors) -> str:
    t = next((x for x in tensors if x is not None), None)
    return f"{op}{tuple(t.shape) if t is not None else ()}"


class Transport:
    kind = "base"
    rank = 0
    size = 1
    group = None

    def global_rank(self, r: int) -> int:
        """Global rank of group rank ``r``."""
        if self.group is None or not dist.is_initialized():
            return r
        return dist.get_global_rank(self.group, r)

    def all_reduce(self, t, async_op=False) -> Handle:
        raise NotImplementedError

    def reduce_scatter(self, out, inp, async_op=False) -> Handle:
        raise NotImplementedError

    def all_gather(self, out, inp, async_op=False) -> Handle:
        raise NotImplementedError

    def broadcast(self, t, src: int, async_op=False) -> Handle:
        """``src`` is a rank of this transport's group."""
        raise NotImplementedError

    def sendrecv(self, sends=(), recvs=(), async_op=False) -> Handle:
        """One grouped exchange: ``sends`` / ``recvs`` are (tensor, peer group rank) pairs."""
        raise NotImplementedError

    def capturable(self) -> bool:
        """Whether the collectives may be recorded into a HIP graph."""
        return False

    @property
    def active(self) -> bool:
        """Whether collectives are issued at all (a native communicator of one rank still
        issues them -- the single-GPU tests of the RCCL path)."""
        return self.size > 1


class TorchTransport(Transport):
    kind = "torch"

    def __init__(self, group=None):
        self.group = group
        self.rank = comm.rank(group)
        self.size = comm.world_size(group)
        # gloo's send/recv take host memory only: a GPU run rehearsed over gloo (several
        # ranks on one device) stages point-to-point payloads through the host
        self.host_staged = dist.is_initialized() and dist.get_backend(group) == "gloo"

    def _ret(self, work, async_op, desc="collective"):
        if async_op:
            return _WorkHandle(work)._track(desc)
        if work is not None:
            work.wait()
        return _Done()

    def all_reduce(self, t, async_op=False):
        if self.size == 1:
            return _Done()
        return self._ret(comm.all_reduce(t, group=self.group, async_op=async_op), async_op,
                         _desc("all_reduce", (t,)))

    def reduce_scatter(self, out, inp, async_op=False):
        if self.size == 1:
            out.copy_(inp)
            return _Done()
        return self._ret(comm.reduce_scatter_into(out, inp, group=self.group, async_op=async_op), async_op,
                         _desc("reduce_scatter", (out,)))

    def all_gather(self, out, inp, async_op=False):
        if self.size == 1:
            out.copy_(inp)
            return _Done()
        return self._ret(comm.all_gather_into(out, inp, group=self.group, async_op=async_op), async_op,
                         _desc("all_gather", (out,)))

    def broadcast(self, t, src, async_op=False):
        if self.size == 1:
            return _Done()
        return self._ret(comm.broadcast(t, src=self.global_rank(src), group=self.group, async_op=async_op),
                         async_op, _desc("broadcast", (t,)))

    def sendrecv(self, sends=(), recvs=(), async_op=False):
        if not sends and not recvs:
            return _Done()
        ops, staged = [], []
        for t, peer in sends:
            t = t.detach().contiguous()
            ops.append(dist.P2POp(dist.isend, t.cpu() if self.host_staged and t.is_cuda else t,
                                  self.global_rank(peer), self.group))
        for t, peer in recvs:
            buf = t
            if self.host_staged and t.is_cuda:
                buf = torch.empty(t.shape, dtype=t.dtype)
                staged.append((t, buf))
            ops.append(dist.P2POp(dist.irecv, buf, self.global_rank(peer), self.group))
        works = dist.batch_isend_irecv(ops)

        def unstage():
            for dst, src in staged:
                dst.copy_(src)

        h = _WorkHandle(works, after=unstage if staged else None)._track(
            _desc("sendrecv", [t for t, _ in sends] + [t for t, _ in recvs]))
        if not async_op:
            h.wait()
            return _Done()
        return h


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def check_peer_comms() -> None:
    """Raise if a peer-access (IPC) communicator's wait gave up since the last check: its data is
    not valid.  Host-synchronous (one read of each error word): called at the trainer's progress
    points and at shutdown."""
    for nc in _native_comms:
        chk = getattr(nc, "check", None)
        if chk is not None and getattr(nc, "_own", None):
            chk()


def shutdown_native() -> None:
    """Destroy every native communicator (splits first) and stop the watchdog: the native
    half of the reference's ``destroy_process_group`` (``/root/reference/main-ddp.py:34-35``).
    Pending collectives are drained first."""
    if not _native_comms:
        return
    from . import native_comm

    if torch.cuda.is_available():
        torch.cuda.synchronize()
    try:
        check_peer_comms()
    except RuntimeError as exc:  # (teardown goes on; the run already produced its output)
        print(f"[comm] {exc}")
    native_comm.watchdog_stop()
    while _native_comms:
        nc = _native_comms.pop()
        try:
            nc.destroy()
        except Exception as exc:  # noqa: BLE001 -- teardown goes on for the others
            print(f"[comm] ncclCommDestroy failed: {exc}")


class NativeTransport(Transport):
    kind = "native"

    def __init__(self, group=None, device=None, native=None):
        from .native_comm import NativeComm

        self.group = group
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type == "cuda" and self.device.index is None:  # ("cuda": the current device)
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.nc = native if native is not None else NativeComm(group, device=self.device)
        self.rank, self.size = self.nc.rank, self.nc.size
        _native_comms.append(self.nc)
        # RCCL runs on its own high-priority stream, ordered with events (a CPU "device" is the
        # host-side fake library of the CPU tests: calls go straight through)
        self.stream = torch.cuda.Stream(device=self.device, priority=-1) if self.device.type == "cuda" else None
        _fake_sink_for(self.device)

    def capturable(self) -> bool:
        return True

    @property
    def active(self) -> bool:
        return True

    def _enqueue(self, fn, tensors, async_op, op="collective"):
        if _STREAM_CHECK:
            for t in tensors:
                if not t.is_contiguous() or t.device != self.device:
                    raise RuntimeError(f"stream-order check: {op} buffer {tuple(t.shape)} on {t.device} "
                                       f"(contiguous={t.is_contiguous()}) handed to the comm stream of {self.device}")
        capturing = _capturing()
        if comm.coll_check_enabled() and not capturing and op != "sendrecv":
            # --coll_check on the production path: every rank's (sequence, op, shape, dtype).
            # Point-to-point exchanges are not lockstep over the group (1F1B posts M exchanges
            # on the first stage, M + 1 on the last, other counts in between), so a group-wide
            # fingerprint would pair up wrongly: skipped, as TorchTransport.sendrecv does
            comm.fingerprint(op, tensors[0] if tensors else None, self.group)
        desc = _desc(op, tensors)
        with mark(f"comm:{op}"):
            return self._launch(fn, tensors, async_op, desc, capturing)

    def _launch(self, fn, tensors, async_op, desc, capturing):
        from . import native_comm

        s = self.stream
        if s is None:  # host-side fake library
            fn(0)
            native_comm.watchdog_track(0, desc)
            return _Done()
        cur = torch.cuda.current_stream(self.device)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            fn(s)
            if _FAKE_COLL and tensors:
                _fake_coll(desc.split("(")[0].split(" ")[0], tensors, s)
        for t in tensors:
            t.record_stream(s)
        done = torch.cuda.Event()
        done.record(s)
        if not capturing:  # (a replayed graph is watched as a whole: GraphedStep)
            native_comm.watchdog_track(s.cuda_stream, desc)
        if async_op:
            _reserve_begin()
        h = _EventHandle(done, reserved=async_op)._track(desc)
        if not async_op:
            h.wait()
            return _Done()
        return h

    def all_reduce(self, t, async_op=False):
        return self._enqueue(lambda s: self.nc.all_reduce(t, stream=s), (t,), async_op, "all_reduce")

    def reduce_scatter(self, out, inp, async_op=False):
        return self._enqueue(lambda s: self.nc.reduce_scatter(out, inp, stream=s), (out, inp), async_op,
                             "reduce_scatter")

    def all_gather(self, out, inp, async_op=False):
        return self._enqueue(lambda s: self.nc.all_gather(out, inp, stream=s), (out, inp), async_op,
                             "all_gather")

    def broadcast(self, t, src, async_op=False):
        return self._enqueue(lambda s: self.nc.broadcast(t, src=src, stream=s), (t,), async_op, "broadcast")

    def sendrecv(self, sends=(), recvs=(), async_op=False):
        if not sends and not recvs:
            return _Done()
        sends = [(t.detach().contiguous(), p) for t, p in sends]

        def run(s):
            with self.nc.grouped():
                for t, p in sends:
                    self.nc.send(t, p, stream=s)
                for t, p in recvs:
                    self.nc.recv(t, p, stream=s)

        return self._enqueue(run, [t for t, _ in sends] + [t for t, _ in recvs], async_op, "sendrecv")

    def split(self, color: int, key: int, group=None) -> "NativeTransport":
        """Sub-communicator (ncclCommSplit) of the ranks sharing ``color``; ``group`` is the
        matching torch group (bootstrap / host-side reductions).  Collective."""
        return NativeTransport(group, self.device, native=self.nc.split(color, key))


class IpcTransport(NativeTransport):
    """Intra-node collectives by direct peer access (``parallel/ipc_comm.py``, ``--comm ipc``):
    the same side-stream / event / watchdog plumbing as the RCCL transport, the kernels of
    ``ops/csrc/ipc_coll.hip`` instead of RCCL's -- all-reduce, reduce-scatter, all-gather,
    broadcast and grouped point-to-point, so every recipe runs on it.  Bootstraps over any process
    group -- gloo included -- so several ranks may share one GPU."""

    kind = "ipc"

    def __init__(self, group=None, device=None):
        from .ipc_comm import IpcComm

        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if dev.type == "cuda" and dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        super().__init__(group, dev, native=IpcComm(group, dev))

    def sendrecv(self, sends=(), recvs=(), async_op=False):
        if not sends and not recvs:
            return _Done()
        sends = [(t.detach().contiguous(), p) for t, p in sends]
        return self._enqueue(lambda s: self.nc.sendrecv(sends, recvs, stream=s),
                             [t for t, _ in sends] + [t for t, _ in recvs], async_op, "sendrecv")

    def split(self, color: int, key: int, group=None):
        raise NotImplementedError("IpcTransport: no sub-communicators (make_mesh_transports builds one per group)")


def _want_native(kind: str, device) -> bool:
    if kind == "torch":
        return False
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if dev.type == "cpu":
        # `--comm native` on CPU runs only against a host-side RCCL stand-in named by
        # DPC_RCCL_LIB (tests/fakes/fake_rccl_hip.cpp, which moves host buffers between the
        # ranks): the CPU tests drive the production transport's multi-rank code through it
        return kind == "native" and bool(os.environ.get("DPC_RCCL_LIB")) and dist.is_initialized()
    return (dev.type == "cuda" and dist.is_initialized() and dist.get_backend() == "nccl")


def make_transport(group=None, device=None, kind: str | None = None) -> Transport:
    """The engines' transport over ``group``: ``kind`` = auto (native on a GPU with the
    nccl backend, torch otherwise) | native | torch.  Falls back to torch -- before any
    collective -- if the native communicator cannot be built."""
    kind = kind or os.environ.get("DPC_COMM", "auto")
    if kind == "ipc" and torch.device(device if device is not None else "cpu").type == "cuda" and dist.is_initialized():
        return IpcTransport(group, device)  # (no fallback: asked for by name)
    if (comm.world_size(group) > 1 or kind == "native") and _want_native(kind, device):
        try:
            return NativeTransport(group, device)
        except Exception as exc:  # library / RCCL missing: stay correct, say so
            if comm.rank() == 0:
                print(f"[comm] native RCCL transport unavailable ({exc}); using torch.distributed")
    return TorchTransport(group)


def make_mesh_transports(pp_group, dp_group, stage: int, replica: int, device=None, kind: str | None = None):
    """(pp, dp) transports of a rank on the 2-D mesh (rank = stage * dp + replica).  Native:
    ONE world communicator split twice with ncclCommSplit (color = replica -> the pipeline of
    this replica, color = stage -> the replicas of this stage)."""
    kind = kind or os.environ.get("DPC_COMM", "auto")
    if kind == "ipc" and comm.world_size() > 1 and torch.device(device if device is not None else "cpu").type == "cuda":
        # one peer-access communicator per group (they bootstrap over any torch group: no split)
        return IpcTransport(pp_group, device), IpcTransport(dp_group, device)
    if comm.world_size() > 1 and _want_native(kind, device):
        built = []
        try:
            world = NativeTransport(None, device)
            built.append(world)
            pp = world.split(replica, stage, group=pp_group)
            built.append(pp)
            dp = world.split(stage, replica, group=dp_group)
            return pp, dp
        except Exception as exc:
            # every bring-up step is agreed (native_comm._agree): all ranks land here together
            for t in reversed(built):
                if t.nc in _native_comms:
                    _native_comms.remove(t.nc)
                t.nc.destroy()
            if comm.rank() == 0:
                print(f"[comm] native RCCL mesh unavailable ({exc}); using torch.distributed")
    return TorchTransport(pp_group), TorchTransport(dp_group)
