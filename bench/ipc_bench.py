"""Peer-access all-reduce (parallel/ipc_comm.py) timing, two ranks sharing ONE GPU: every byte
then moves through the same HBM, so this measures the kernel's latency floor (flag barriers
through uncached memory, the launch) and its local-copy rate -- not xGMI.  Rank 0 prints one
JSON line per size.

    python bench/ipc_bench.py            # spawns the two ranks itself (gloo bootstrap)
"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rank(rank, world, port, sizes, iters):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DPC_DIST_BACKEND="gloo")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist

    from distributed_pytorch_cookbook_amd.parallel import comm
    from distributed_pytorch_cookbook_amd.parallel.ipc_comm import IpcComm

    comm.init_dist()
    c = IpcComm(slot_mb=256)
    for nbytes in sizes:
        n = nbytes // 4
        t = torch.ones(n, device="cuda")
        for _ in range(3):
            c.all_reduce(t)
        torch.cuda.synchronize()
        dist.barrier()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            c.all_reduce(t)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / iters
        c.check()
        ms = torch.tensor([us])
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        if rank == 0:
            print(json.dumps({"bytes": nbytes, "us": round(float(ms), 2),
                              "algbw_GBps": round(nbytes / float(ms) / 1e3, 1)}), flush=True)
    c.destroy()
    dist.destroy_process_group()


def main():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from dist_helpers import free_port

    sizes = [4096, 65536, 1 << 20, 16 << 20, 128 << 20]
    mp.spawn(_rank, args=(2, free_port(), sizes, 20), nprocs=2, join=True)


if __name__ == "__main__":
    main()
