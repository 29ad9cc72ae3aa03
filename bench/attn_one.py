"""Run the attention kernels repeatedly (for rocprofv3 PMC / kernel-trace).

    python bench/attn_one.py --N 32 --S 1023 --H 12 --iters 5 [--bwd]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.environ.get("DPC_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops.attention import attention_bwd, attention_fwd  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--N", type=int, default=32)
ap.add_argument("--S", type=int, default=1023)
ap.add_argument("--H", type=int, default=12)
ap.add_argument("--iters", type=int, default=5)
ap.add_argument("--bwd", action="store_true")
ap.add_argument("--hd", type=int, default=64)
a = ap.parse_args()
hd = a.hd
qkv = torch.randn(a.N * a.S, 3 * a.H * hd, device="cuda").bfloat16()
o, lse = attention_fwd(qkv, a.N, a.S, a.H, hd)
do = torch.randn(a.N * a.S, a.H * hd, device="cuda").bfloat16()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(a.iters):
    if a.bwd:
        attention_bwd(do, qkv, o, lse, a.N, a.S, a.H, hd)
    else:
        attention_fwd(qkv, a.N, a.S, a.H, hd)
e.record()
torch.cuda.synchronize()
fl = 4 * a.N * a.H * a.S * a.S * hd / 2 * (2.5 if a.bwd else 1.0)
ms = s.elapsed_time(e) / a.iters
print(f"{'bwd' if a.bwd else 'fwd'} N={a.N} S={a.S} H={a.H} hd={hd}: {ms * 1e3:.1f} us  {fl / ms / 1e9:.1f} TF/s")
