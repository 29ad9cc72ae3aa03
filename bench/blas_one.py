"""Run torch.mm (hipBLASLt) on one shape repeatedly -- for rocprofv3 kernel traces of the vendor
kernel's launch geometry (grid, workgroup, VGPR/AGPR, LDS) next to our own kernels.

    python bench/blas_one.py --M 65472 --N 2304 --K 768 --layout nt
"""
import argparse

import torch

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=65472)
ap.add_argument("--N", type=int, default=2304)
ap.add_argument("--K", type=int, default=768)
ap.add_argument("--layout", default="nt", choices=["nt", "nn"])
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
A = (torch.rand(a.M, a.K, device="cuda") * 2 - 1).bfloat16()
B = (torch.rand(a.N, a.K, device="cuda") * 2 - 1).bfloat16()
if a.layout == "nn":
    B = B.t().contiguous()
for _ in range(a.iters):
    torch.mm(A, B.t() if a.layout == "nt" else B)
torch.cuda.synchronize()
