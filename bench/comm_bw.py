"""Collective bus-bandwidth microbenchmark over RCCL (xGMI) -- SURVEY.md §7.2 step 4.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/comm_bw.py \
        [--sizes_mb 1 8 32 128 512] [--ops all_reduce all_gather reduce_scatter broadcast sendrecv] \
        [--backend torch|native|both] [--dtype fp32|bf16] [--json gpurun_out/comm_bw.json]

One rank per GPU.  Every (op, size) is timed over ``--iters`` back-to-back launches after
warmup, bracketed by device synchronisation, and the MAX over ranks is reported with the
nccl-tests conventions:
  algbw = bytes / time;  busbw = algbw * factor, factor = 2(W-1)/W for all-reduce,
  (W-1)/W for all-gather / reduce-scatter (bytes = the full gathered buffer), 1 for
  broadcast and send/recv (ring neighbour exchange, every rank sends and receives).
``torch`` goes through torch.distributed's nccl (= RCCL) process group; ``native`` through
the framework's C++ RCCL communicator (parallel/native_comm.py) on a dedicated stream.
These are the numbers the DDP bucket size (``--bucket_mb``) and the FSDP unit size are
chosen against: ring collectives over xGMI are per-link bound, so busbw saturates only
for messages of tens of MB and more.  On CPU (gloo, tests) it runs the same loop.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.parallel import comm  # noqa: E402


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def bus_factor(op: str, w: int) -> float:
    if op == "all_reduce":
        return 2.0 * (w - 1) / w
    if op in ("all_gather", "reduce_scatter"):
        return (w - 1) / w
    return 1.0


def make_op(op, nbytes, dtype, dev, w, rank, backend, native):
    esz = torch.tensor([], dtype=dtype).element_size()
    n = max(w, nbytes // esz // w * w)
    if op == "all_reduce":
        t = torch.ones(n, dtype=dtype, device=dev)
        if backend == "native":
            return (lambda: native.all_reduce(t)), n * esz
        return (lambda: dist.all_reduce(t)), n * esz
    if op == "all_gather":
        inp = torch.ones(n // w, dtype=dtype, device=dev)
        out = torch.empty(n, dtype=dtype, device=dev)
        if backend == "native":
            return (lambda: native.all_gather(out, inp)), n * esz
        return (lambda: dist.all_gather_into_tensor(out, inp)), n * esz
    if op == "reduce_scatter":
        inp = torch.ones(n, dtype=dtype, device=dev)
        out = torch.empty(n // w, dtype=dtype, device=dev)
        if backend == "native":
            return (lambda: native.reduce_scatter(out, inp)), n * esz
        return (lambda: dist.reduce_scatter_tensor(out, inp)), n * esz
    if op == "broadcast":
        t = torch.ones(n, dtype=dtype, device=dev)
        if backend == "native":
            return (lambda: native.broadcast(t, 0)), n * esz
        return (lambda: dist.broadcast(t, 0)), n * esz
    if op == "sendrecv":  # ring: send to rank+1, receive from rank-1, all pairs concurrently
        s = torch.ones(n, dtype=dtype, device=dev)
        r = torch.empty(n, dtype=dtype, device=dev)
        nxt, prv = (rank + 1) % w, (rank - 1) % w
        if backend == "native":
            def f():
                with native.grouped():
                    native.send(s, nxt)
                    native.recv(r, prv)
            return f, n * esz

        def g():
            for work in dist.batch_isend_irecv([dist.P2POp(dist.isend, s, nxt), dist.P2POp(dist.irecv, r, prv)]):
                work.wait()
        return g, n * esz
    raise ValueError(op)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes_mb", type=float, nargs="+", default=[1, 8, 32, 128, 512])
    ap.add_argument("--ops", nargs="+", default=["all_reduce", "all_gather", "reduce_scatter", "broadcast",
                                                 "sendrecv"])
    ap.add_argument("--backend", default="torch", choices=["torch", "native", "both"])
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    info = comm.init_dist(force_cpu=a.cpu)
    w, rank, dev = info.world_size, info.rank, info.device
    if w < 2:
        if rank == 0:
            print(json.dumps({"note": "comm_bw needs >= 2 ranks (torchrun --nproc-per-node N)"}))
        return
    dtype = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    backends = ["torch", "native"] if a.backend == "both" else [a.backend]
    native = None
    if "native" in backends:
        if dev.type != "cuda":
            backends = [b for b in backends if b != "native"]
        else:
            from distributed_pytorch_cookbook_amd.parallel.native_comm import NativeComm

            native = NativeComm(None, device=dev)
    rows = []
    for be in backends:
        for op in a.ops:
            for mb in a.sizes_mb:
                fn, nbytes = make_op(op, int(mb * 2**20), dtype, dev, w, rank, be, native)
                for _ in range(a.warmup):
                    fn()
                _sync(dev)
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    fn()
                _sync(dev)
                dt = torch.tensor([(time.perf_counter() - t0) / a.iters], dtype=torch.float64)
                if dev.type == "cuda":
                    dt = dt.to(dev)
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
                t = float(dt.item())
                algbw = nbytes / t / 1e9
                rows.append(dict(backend=be, op=op, bytes=nbytes, dtype=a.dtype, world=w, us=round(t * 1e6, 1),
                                 algbw_GBps=round(algbw, 2), busbw_GBps=round(algbw * bus_factor(op, w), 2)))
                if rank == 0:
                    print(json.dumps(rows[-1]), flush=True)
    if native is not None:
        native.destroy()
    if rank == 0 and a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)
    comm.cleanup_dist()


if __name__ == "__main__":
    main()
