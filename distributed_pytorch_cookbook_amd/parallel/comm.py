"""Process-group bring-up and small collective helpers.

Reference: ``init_mp`` / ``cleanup_mp`` (``/root/reference/main-ddp.py:25-35``,
``main-fsdp.py:29-39``): ``init_process_group("nccl")`` and ``cuda:{rank % ngpu}``.
Here: one process per GPU bound by ``LOCAL_RANK`` (torchrun), backend ``nccl`` -- which
on ROCm *is* RCCL over xGMI -- on a HIP device, ``gloo`` on CPU (tests), and 2-D
sub-groups for the PP x DP mesh.  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is forced for RCCL's
dmabuf IPC on this platform.

Debug aids:
* ``DPC_COLL_CHECK=1`` -- every engine collective first all-gathers a fingerprint
  (sequence number, op, numel, dtype) and raises on a mismatch, turning a would-be hang
  from unmatched collectives (the reference's rank-0-only FSDP generate,
  ``main-fsdp.py:184-188``) into an immediate error naming both sides.
* ``DPC_COLL_TIMEOUT`` (seconds) -- process-group timeout (watchdog) for hung collectives.
"""
from __future__ import annotations

import datetime
import os
import zlib
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def env_world() -> int:
    return int(os.environ.get("WORLD_SIZE", "1"))


def init_dist(force_cpu: bool = False, force_group: bool = False) -> DistInfo:
    """Initialise the default process group from torchrun's env (no-op for 1 process, unless
    ``force_group``: a 1-rank group on 127.0.0.1 to bootstrap a native communicator)."""
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    world = env_world()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = (not force_cpu) and torch.cuda.is_available()
    if use_gpu:
        ndev = torch.cuda.device_count()
        torch.cuda.set_device(local_rank % ndev)
        device = torch.device("cuda", local_rank % ndev)
    else:
        device = torch.device("cpu")
    backend = "none"
    if world > 1 and not dist.is_initialized():
        backend = "nccl" if use_gpu else "gloo"
        # DPC_DIST_BACKEND=gloo: rehearse the multi-rank GPU path with several ranks on ONE
        # device (RCCL refuses two ranks per GPU); collectives then stage through the host
        backend = os.environ.get("DPC_DIST_BACKEND", backend)
        timeout = datetime.timedelta(seconds=float(os.environ.get("DPC_COLL_TIMEOUT", "1800")))
        kw = dict(backend=backend, timeout=timeout)
        if use_gpu and backend == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    elif force_group and not dist.is_initialized():
        import socket

        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        backend = "nccl" if use_gpu else "gloo"
        kw = dict(backend=backend, init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        if use_gpu:
            kw["device_id"] = device
        dist.init_process_group(**kw)
    elif dist.is_initialized():
        backend = dist.get_backend()
    return DistInfo(rank, world, local_rank, device, backend)


def cleanup_dist() -> None:
    """Reference ``cleanup_mp`` (``/root/reference/main-ddp.py:34-35``): the engines' native
    RCCL communicators are destroyed (and their watchdog stopped) before the process group."""
    from .transport import shutdown_native

    if dist.is_initialized():
        dist.barrier()
    shutdown_native()
    if dist.is_initialized():
        dist.destroy_process_group()


def world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def barrier(group=None) -> None:
    if dist.is_initialized() and world_size(group) > 1:
        dist.barrier(group=group)


# ------------------------------------------------------------------ collective fingerprints
_CHECK = os.environ.get("DPC_COLL_CHECK", "0") == "1"
_seq = {}


def set_coll_check(on: bool) -> None:
    global _CHECK
    _CHECK = bool(on)


def coll_check_enabled() -> bool:
    return _CHECK


def fingerprint(op: str, t: torch.Tensor | None, group) -> None:
    """All-gather this rank's (sequence number, crc32(op, shape, dtype)) for ``group`` and
    raise on any mismatch (``--coll_check``; used by both transports)."""
    _fingerprint(op, t, group)


def _fingerprint(op: str, t: torch.Tensor | None, group) -> None:
    if not _CHECK or not dist.is_initialized():
        return
    key = id(group)
    _seq[key] = _seq.get(key, 0) + 1
    desc = f"{op}:{tuple(t.shape) if t is not None else ()}:{t.dtype if t is not None else None}"
    fp = torch.tensor([_seq[key], zlib.crc32(desc.encode())], dtype=torch.int64)
    dev = t.device if (t is not None and t.is_cuda) else torch.device("cpu")
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    fp = fp.to(dev)
    out = [torch.empty_like(fp) for _ in range(world_size(group))]
    dist.all_gather(out, fp, group=group)
    vals = [tuple(o.tolist()) for o in out]
    if len(set(vals)) != 1:
        raise RuntimeError(f"collective mismatch at #{_seq[key]} ({desc}) across ranks: {vals}")


def all_reduce(t, op=dist.ReduceOp.SUM, group=None, async_op=False):
    _fingerprint("all_reduce", t, group)
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


def broadcast(t, src, group=None, async_op=False):
    _fingerprint("broadcast", t, group)
    return dist.broadcast(t, src=src, group=group, async_op=async_op)


def all_gather_into(out, inp, group=None, async_op=False):
    _fingerprint("all_gather", inp, group)
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def reduce_scatter_into(out, inp, op=dist.ReduceOp.SUM, group=None, async_op=False):
    _fingerprint("reduce_scatter", out, group)
    return dist.reduce_scatter_tensor(out, inp, op=op, group=group, async_op=async_op)


def gather_objects(obj):
    """Every rank's ``obj`` as a list indexed by rank (a single-element list without a
    process group).  Collective: call on every rank."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def all_reduce_scalars(values: list[float | torch.Tensor], device, group=None, op="sum"):
    """Reduce several scalars in ONE collective (reference issues one per metric,
    main-ddp.py:159-160)."""
    t = torch.stack([torch.as_tensor(v).detach().to(device=device, dtype=torch.float32).reshape(())
                     for v in values])
    if world_size(group) > 1:
        all_reduce(t, dist.ReduceOp.SUM, group)
        if op == "mean":
            t /= world_size(group)
    return t


def make_mesh(pp: int, dp: int):
    """2-D (pp, dp) mesh over the default group: rank = stage * dp + replica.

    Returns (pp_group_of_this_rank, dp_group_of_this_rank, stage, replica, pp_ranks).
    Every rank creates every group (torch requirement)."""
    world = world_size()
    assert pp * dp == world, f"pp({pp}) x dp({dp}) != world({world})"
    r = rank()
    stage, replica = r // dp, r % dp
    my_pp, my_dp = None, None
    pp_ranks = None
    for rep in range(dp):
        ranks = [s * dp + rep for s in range(pp)]
        g = dist.new_group(ranks) if world > 1 else None
        if rep == replica:
            my_pp, pp_ranks = g, ranks
    for s in range(pp):
        ranks = [s * dp + rep for rep in range(dp)]
        g = dist.new_group(ranks) if world > 1 else None
        if s == stage:
            my_dp = g
    return my_pp, my_dp, stage, replica, pp_ranks
