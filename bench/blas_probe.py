"""Run hipBLASLt (torch.mm) on the GPT-2-small products so a rocprofv3 kernel trace shows the
library's kernel choice per shape (name = macro tile, waves, grid, LDS, VGPRs).

    rocprofv3 --kernel-trace -f csv -d DIR -o b -- python bench/blas_probe.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.gemm_ab import GPT2S, operands, torch_fn  # noqa: E402

for name, M, N, K, lay in GPT2S + [("sq8k_nt", 8192, 8192, 8192, "nt")]:
    A, B, _, odt = operands(M, N, K, lay)
    out = torch.empty(M, N, device="cuda", dtype=odt)
    f = torch_fn(A, B, lay, out)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    print(name, flush=True)
