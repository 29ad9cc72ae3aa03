"""Multi-process CPU (gloo) harness for the parallel engines."""
from __future__ import annotations

import os
import socket
import sys
import traceback

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(rank, world, port, fn, args, errq):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    torch.set_num_threads(1)
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    try:
        fn(rank, world, *args)
    except Exception:  # pragma: no cover - surfaced by the parent
        errq.put((rank, traceback.format_exc()))
        raise
    finally:
        import torch.distributed as dist

        if dist.is_initialized():
            dist.destroy_process_group()


def _run_once(fn, world: int, args, timeout: float):
    import time

    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, errq)) for r in range(world)]
    for p in procs:
        p.start()
    errs = []
    deadline = time.monotonic() + timeout
    # poll: a rank that fails (e.g. the rendezvous port taken) must not leave its peers waiting
    # for it until the timeout
    while any(p.is_alive() for p in procs) and time.monotonic() < deadline:
        while not errq.empty():
            errs.append(errq.get())
        if errs:
            break
        time.sleep(0.05)
    for p in procs:
        p.join(0 if errs else 1.0)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join(5)
    while not errq.empty():
        errs.append(errq.get())
    return procs, alive, errs


def run_workers(fn, world: int, *args, timeout: float = 240.0):
    for attempt in range(3):
        procs, alive, errs = _run_once(fn, world, args, timeout)
        # the free port can be taken between free_port() and the rendezvous: try another one
        if errs and attempt < 2 and any("EADDRINUSE" in tb or "address already in use" in tb for _, tb in errs):
            continue
        break
    if errs:
        raise AssertionError("worker failure:\n" + "\n".join(f"[rank {r}]\n{tb}" for r, tb in errs))
    if alive:
        raise AssertionError(f"{len(alive)} worker(s) hung (killed after {timeout}s)")
    bad = [p.exitcode for p in procs if p.exitcode != 0]
    if bad:
        raise AssertionError(f"worker exit codes {bad}")
