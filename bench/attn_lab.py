"""Per-workgroup cost ablations of the attention backward kernels (GPT-2 small shape).

    python bench/attn_lab.py [--N 64 --S 1023 --H 12] [--rounds 5 --iters 10]

Times the delta pre-pass, and the dK/dV and dQ kernels of the shipped hd-64 variant with the
compile-time ablation bits of ``dpc_attn_bwd_lab`` (attention.hip): 1 = no tile loop, 2 = no
per-row register loads, 4 = no epilogue stores, 8 = no ring prologue.  Variants interleave in
rounds inside one process (median).  Ablated outputs are wrong by design.
"""
from __future__ import annotations

import argparse
import ctypes
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.attention import attention_fwd, split_qkv  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--N", type=int, default=64)
ap.add_argument("--S", type=int, default=1023)
ap.add_argument("--H", type=int, default=12)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
hd, N, S, H = 64, a.N, a.S, a.H
T = N * S
qkv = torch.randn(T, 3 * H * hd, device="cuda").bfloat16()
o, lse = attention_fwd(qkv, N, S, H, hd)
do = torch.randn(T, H * hd, device="cuda").bfloat16()
dqkv = torch.empty_like(qkv)
delta = torch.empty(2, N * H, S, device="cuda", dtype=torch.float32)
q, k, v = split_qkv(qkv, H, hd)
dq, dk, dv = split_qkv(dqkv, H, hd)
args = _lib.AttnArgs(q=q.data_ptr(), k=k.data_ptr(), v=v.data_ptr(), o=o.data_ptr(), lse=lse.data_ptr(),
                     pad=None, dout=do.data_ptr(), dq=dq.data_ptr(), dk=dk.data_ptr(), dv=dv.data_ptr(),
                     delta=delta.data_ptr(), ld_qkv=qkv.stride(0), ld_o=o.stride(0), ld_dqkv=dqkv.stride(0),
                     N=N, S=S, H=H, scale=1.0 / math.sqrt(hd), causal=1, hd=hd)
lib = _lib.lib()
fn = lib.dpc_attn_bwd_lab
fn.argtypes = [ctypes.POINTER(_lib.AttnArgs), ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
fn.restype = ctypes.c_int
stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run(which, abl):
    rc = fn(ctypes.byref(args), which, abl, stream)
    if rc != 0:
        raise RuntimeError(f"dpc_attn_bwd_lab({which}, {abl}) -> {rc}")


variants = [("pre", 0, 0)]
names = {0: "full", 1: "no_loop", 2: "no_rowload", 4: "no_store", 6: "no_rowload_no_store",
         3: "no_loop_no_rowload", 5: "no_loop_no_store", 7: "prologue_only", 15: "empty"}
for which, kname in ((1, "dkdv"), (2, "dq")):
    for abl in (0, 2, 4, 6, 1, 3, 5, 7, 15):
        variants.append((f"{kname}_{names[abl]}", which, abl))
run(0, 0)
for _, w, b in variants:
    run(w, b)
torch.cuda.synchronize()
times = {v[0]: [] for v in variants}
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(a.rounds):
    for name, w, b in variants:
        ev0.record()
        for _ in range(a.iters):
            run(w, b)
        ev1.record()
        ev1.synchronize()
        times[name].append(ev0.elapsed_time(ev1) / a.iters * 1e3)
for name, _, _ in variants:
    xs = times[name]
    print(f"{name:28s} median {statistics.median(xs):8.1f} us  min {min(xs):8.1f}", flush=True)
