"""Intra-node collectives by direct peer access (``ops/csrc/ipc_coll.hip``), SURVEY.md §5.8.

Every rank allocates a staging buffer (two halves, used alternately) and an uncached flag
array, exports both through HIP IPC, and maps every other rank's; the handles travel over
the bootstrap process group (``all_gather_object``).  A collective is then ONE kernel on the
caller's stream: the two-shot all-reduce reads each shard straight out of the peers' HBM over
their xGMI links (reduce-scatter, then all-gather of the summed shards), so all 7 links of an
8-GPU node carry traffic at once instead of a ring's one.  No host synchronisation and no
per-call host state (the epoch counters live in device memory), so a HIP graph captures the
collectives of a step and every replay runs them afresh.

It is also what lets ONE GPU rehearse the N > 1 step graph: RCCL refuses two ranks on one
device ("Duplicate GPU detected"), HIP IPC does not, so ``IpcTransport`` runs DDP / FSDP at
world 2 on one MI355X with the step captured on both ranks (``tests/test_ipc_gpu.py``).

Results are bitwise identical on every rank (each shard is summed once, in rank order, by its
owner).  Collectives larger than a staging half are chunked.  A wait that never completes --
a peer that crashed or took another code path -- sets the error word after ``spin_limit``
polls instead of hanging the GPU; ``check()`` raises on it.
"""
from __future__ import annotations

import contextlib
import ctypes
import os

import torch
import torch.distributed as dist

ALLREDUCE, REDUCE_SCATTER, ALLGATHER, BROADCAST = 0, 1, 2, 3
_ALIGN = 64  # elements (ipc_coll.hip: IPC_ALIGN)


def _lib():
    from ..ops import _lib as L

    return L.lib()


def _rc(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: hipError {rc}")


class IpcComm:
    """Peer-access communicator over the ranks of ``group`` (all on one node, ``world <= 8``).

    ``slot_mb``: one staging half in MiB (DPC_IPC_SLOT_MB, default 64); the buffer holds two.
    ``p2p_mb``: one point-to-point channel buffer in MiB (DPC_IPC_P2P_MB, default 16; 2 x world
    of them per rank, 0 = no point-to-point)."""

    def __init__(self, group=None, device=None, slot_mb: float | None = None, spin_limit: int | None = None,
                 p2p_mb: float | None = None):
        from ..ops import _lib as L

        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.size = dist.get_world_size(group) if dist.is_initialized() else 1
        if self.size > L.IPC_MAXW:
            raise ValueError(f"IpcComm: {self.size} ranks, at most {L.IPC_MAXW} (one node)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        slot_mb = float(os.environ.get("DPC_IPC_SLOT_MB", "64")) if slot_mb is None else slot_mb
        self.half_bytes = max(256, int(slot_mb * 2**20) // 256 * 256)
        p2p_mb = float(os.environ.get("DPC_IPC_P2P_MB", "16")) if p2p_mb is None else p2p_mb
        self.region_bytes = int(p2p_mb * 2**20) // 256 * 256 if self.size > 1 else 0
        # ~2^26 polls with a short sleep each: tens of seconds before a wait gives up
        self.spin_limit = int(os.environ.get("DPC_IPC_SPIN", str(1 << 26))) if spin_limit is None else spin_limit
        lib = _lib()
        self.groups = lib.dpc_ipc_groups()
        hsize = lib.dpc_ipc_handle_size()
        with torch.cuda.device(self.device):
            # staging (collectives), flag arrays ([0] barriers, [1] p2p READY, [2] p2p ACK: uncached),
            # p2p channel buffers (2 halves x world regions)
            sizes = [(2 * self.half_bytes, 0), (3 * L.IPC_MAXW * self.groups * 4, 1)]
            if self.region_bytes:
                sizes.append((2 * self.size * self.region_bytes, 0))
            own, raws = [], []
            for nbytes, uncached in sizes:
                ptr, h = ctypes.c_void_p(), ctypes.create_string_buffer(hsize)
                _rc(lib.dpc_ipc_alloc(nbytes, uncached, ctypes.byref(ptr)), "IPC buffer allocation")
                own.append(ptr.value)
                _rc(lib.dpc_ipc_handle(ptr, h), "hipIpcGetMemHandle")
                raws.append(h.raw)
            self._own = tuple(own)
            torch.cuda.synchronize(self.device)  # (the allocations' zero fill done before any peer maps them)
            handles = [None] * self.size
            if self.size > 1:
                dist.all_gather_object(handles, tuple(raws), group=group)
            else:
                handles[0] = tuple(raws)
            self.slots = [0] * L.IPC_MAXW
            self.flags = [0] * L.IPC_MAXW
            self.p2p_slots = [0] * L.IPC_MAXW
            tables = (self.slots, self.flags, self.p2p_slots)
            self._opened = []
            err = None
            try:
                for p in range(self.size):
                    if p == self.rank:
                        for tab, v in zip(tables, self._own):
                            tab[p] = v
                        continue
                    for tab, raw in zip(tables, handles[p]):
                        out = ctypes.c_void_p()
                        _rc(lib.dpc_ipc_open(ctypes.create_string_buffer(raw, hsize), ctypes.byref(out)),
                            f"hipIpcOpenMemHandle (rank {p})")
                        self._opened.append(out.value)
                        tab[p] = out.value
            except RuntimeError as exc:
                err = exc
            # every rank mapped every peer, or all of them give up together (no rank left waiting in
            # a barrier for one that raised)
            from .native_comm import _agree

            if not _agree(err is None, group):
                self._release_buffers()
                raise RuntimeError(f"IpcComm: peer buffers could not be mapped on every rank ({err or 'another rank'})")
            self.ep = torch.zeros(self.groups, dtype=torch.int32, device=self.device)
            self.p2p_cnt = torch.zeros(2 * L.IPC_MAXW * self.groups, dtype=torch.int32, device=self.device)
            self.error = torch.zeros(1, dtype=torch.int32, device=self.device)
        if self.size > 1:
            dist.barrier(group=group)  # every rank mapped every buffer before any collective

    # ------------------------------------------------------------------ collectives
    def _launch(self, op, inp, out, n, bf16, root=0, stream=None):
        from ..ops import _lib as L

        a = L.IpcCollArgs()
        for p in range(L.IPC_MAXW):
            a.slot[p] = self.slots[p] or None
            a.flags[p] = self.flags[p] or None
        a.ep, a.error = self.ep.data_ptr(), self.error.data_ptr()
        a.inp, a.out = inp, out
        a.n, a.half_bytes, a.spin_limit = int(n), self.half_bytes, self.spin_limit
        a.op, a.bf16, a.rank, a.world, a.root = op, int(bf16), self.rank, self.size, int(root)
        s = (stream or torch.cuda.current_stream(self.device)).cuda_stream
        _rc(_lib().dpc_ipc_coll(ctypes.byref(a), s), "dpc_ipc_coll")

    def _cap(self, op, es):
        """Elements per chunk that fit one staging half."""
        W = self.size
        per = self.half_bytes // es
        if op == ALLREDUCE:  # n <= W x (largest padded shard that fits)
            return W * (per // W // _ALIGN * _ALIGN)
        if op == REDUCE_SCATTER:
            return per // W // _ALIGN * _ALIGN
        return per // _ALIGN * _ALIGN

    @staticmethod
    def _on(stream):
        """The collective's stream as the current one (the chunked paths' staging tensors are
        allocated, filled and read there, in order with the kernels)."""
        return torch.cuda.stream(stream) if stream is not None else contextlib.nullcontext()

    @staticmethod
    def _kind(t):
        if t.dtype == torch.float32:
            return False, 4
        if t.dtype == torch.bfloat16:
            return True, 2
        raise TypeError(f"IpcComm: {t.dtype} (sums in f32 and bf16 only)")

    @staticmethod
    def _raw(t):
        """A tensor of any dtype as 2-byte units for the copy-only collectives (broadcast,
        all-gather): the kernel moves their bits without arithmetic."""
        if t.dtype in (torch.float32, torch.bfloat16):
            return t
        flat = t.reshape(-1)
        if (flat.numel() * flat.element_size()) % 2:
            raise TypeError(f"IpcComm: {t.dtype} x {flat.numel()} is an odd number of bytes")
        return flat.view(torch.uint8).view(torch.bfloat16) if flat.element_size() == 1 else flat.view(torch.bfloat16)

    def all_reduce(self, t, stream=None):
        """Sum over the ranks, in place."""
        bf, es = self._kind(t)
        flat = t.view(-1)
        n, cap = flat.numel(), self._cap(ALLREDUCE, es)
        for c0 in range(0, n, cap):
            c1 = min(n, c0 + cap)
            p = flat[c0:c1].data_ptr()
            self._launch(ALLREDUCE, p, p, c1 - c0, bf, stream=stream)

    def reduce_scatter(self, out, inp, stream=None):
        """out = sum over ranks of inp[rank * n : (rank + 1) * n], n = out.numel()."""
        bf, es = self._kind(out)
        n, W = out.numel(), self.size
        if inp.numel() != W * n or inp.dtype != out.dtype:
            raise ValueError("reduce_scatter: inp must hold world x out elements of out's dtype")
        cap = self._cap(REDUCE_SCATTER, es)
        if n <= cap:
            self._launch(REDUCE_SCATTER, inp.data_ptr(), out.data_ptr(), n, bf, stream=stream)
            return
        # chunked: shard s of chunk k = inp[s n + k cap ...]: gather those pieces per chunk (the
        # staging copies on the collective's stream, ordered with its kernels)
        iv = inp.view(W, n)
        with self._on(stream):
            for c0 in range(0, n, cap):
                c1 = min(n, c0 + cap)
                piece = iv[:, c0:c1].contiguous()
                self._launch(REDUCE_SCATTER, piece.data_ptr(), out.view(-1)[c0:c1].data_ptr(), c1 - c0, bf,
                             stream=stream)

    def all_gather(self, out, inp, stream=None):
        """out[rank * n : (rank + 1) * n] = inp of every rank, n = inp.numel() (any dtype)."""
        if out.dtype != inp.dtype:
            raise ValueError("all_gather: out and inp dtypes differ")
        out, inp = self._raw(out), self._raw(inp)
        bf, es = self._kind(inp)
        n, W = inp.numel(), self.size
        if out.numel() != W * n or inp.dtype != out.dtype:
            raise ValueError("all_gather: out must hold world x inp elements of inp's dtype")
        cap = self._cap(ALLGATHER, es)
        if n <= cap:
            self._launch(ALLGATHER, inp.data_ptr(), out.data_ptr(), n, bf, stream=stream)
            return
        ov = out.view(W, n)
        with self._on(stream):
            for c0 in range(0, n, cap):
                c1 = min(n, c0 + cap)
                piece = torch.empty((W, c1 - c0), dtype=out.dtype, device=out.device)
                self._launch(ALLGATHER, inp.view(-1)[c0:c1].data_ptr(), piece.data_ptr(), c1 - c0, bf, stream=stream)
                ov[:, c0:c1].copy_(piece)

    def broadcast(self, t, src: int = 0, stream=None):
        """``t`` of rank ``src`` to every rank, in place (any dtype)."""
        t = self._raw(t)
        bf, es = self._kind(t)
        flat = t.view(-1)
        n, cap = flat.numel(), self._cap(BROADCAST, es)
        for c0 in range(0, n, cap):
            c1 = min(n, c0 + cap)
            p = flat[c0:c1].data_ptr()
            self._launch(BROADCAST, p, p, c1 - c0, bf, root=src, stream=stream)

    def sendrecv(self, sends=(), recvs=(), stream=None):
        """One grouped exchange: ``sends`` / ``recvs`` are (tensor, peer group rank) pairs; messages
        on one channel are received in the order they were sent.  Messages larger than a channel
        buffer go in pieces, piece i of every message in the i-th kernel (both sides derive the
        same split from the message sizes)."""
        from ..ops import _lib as L

        if not sends and not recvs:
            return
        if not self.region_bytes:
            raise RuntimeError("IpcComm: point-to-point disabled (p2p_mb = 0) or a one-rank group")
        units = self.region_bytes // 2

        def pieces(t):
            if not t.is_contiguous() or (t.numel() * t.element_size()) % 2:
                raise ValueError("IpcComm.sendrecv: contiguous tensors of an even byte count")
            n = t.numel() * t.element_size() // 2
            base = t.data_ptr()
            return [(base + 2 * u0, min(units, n - u0)) for u0 in range(0, n, units)] or [(base, 0)]

        sp = [(pieces(t), q) for t, q in sends]
        rp = [(pieces(t), q) for t, q in recvs]
        nround = max([len(x) for x, _ in sp + rp])
        s = (stream or torch.cuda.current_stream(self.device)).cuda_stream
        for i in range(nround):
            snd = [(x[i], q) for x, q in sp if i < len(x)]
            rcv = [(x[i], q) for x, q in rp if i < len(x)]
            while snd or rcv:
                a = L.IpcP2PArgs()
                for p in range(L.IPC_MAXW):
                    a.slot[p] = self.p2p_slots[p] or None
                    a.flags[p] = self.flags[p] or None
                a.cnt, a.error = self.p2p_cnt.data_ptr(), self.error.data_ptr()
                a.region_bytes, a.spin_limit = self.region_bytes, self.spin_limit
                a.rank, a.world = self.rank, self.size
                bs, snd = snd[:L.IPC_P2P_MAX], snd[L.IPC_P2P_MAX:]
                br, rcv = rcv[:L.IPC_P2P_MAX], rcv[L.IPC_P2P_MAX:]
                for j, ((ptr, n), q) in enumerate(bs):
                    a.send_ptr[j], a.send_n[j], a.send_peer[j] = ptr, n, q
                for j, ((ptr, n), q) in enumerate(br):
                    a.recv_ptr[j], a.recv_n[j], a.recv_peer[j] = ptr, n, q
                a.nsend, a.nrecv = len(bs), len(br)
                _rc(_lib().dpc_ipc_p2p(ctypes.byref(a), s), "dpc_ipc_p2p")

    # ------------------------------------------------------------------ health / teardown
    def check(self) -> None:
        """Raise if a peer wait timed out (the data of that collective is not valid)."""
        if int(self.error.item()) != 0:
            raise RuntimeError("IpcComm: a peer never reached a collective's barrier (timed out)")

    check_async = check  # (transport.check_drained polls every communicator through this name)

    def _release_buffers(self) -> None:
        lib = _lib()
        for p in self._opened:
            lib.dpc_ipc_close(ctypes.c_void_p(p))
        self._opened = []
        for p in self._own:
            lib.dpc_ipc_free(ctypes.c_void_p(p))
        self._own = ()

    def destroy(self) -> None:
        if not self._own:
            return
        torch.cuda.synchronize(self.device)
        if self.size > 1 and dist.is_initialized():
            dist.barrier(group=self.group)  # no peer still reads this rank's buffers
        self._release_buffers()
