"""Locate non-finite outputs of the v9 forward epilogue (impl 26) on a ragged product: which
tiles (full-tile fast path or the generic edge copy) and which output (C / aux_out)."""
import sys

import torch

sys.path.insert(0, ".")
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402
from distributed_pytorch_cookbook_amd.ops.gemm import gemm  # noqa: E402

torch.manual_seed(3)
M, N, K = 1023, 768, 768
a = torch.randn(M, K, device="cuda").bfloat16()
b = torch.randn(N, K, device="cuda").bfloat16()
bias = torch.randn(N, device="cuda")
for deriv in (False, True):
    for trial in range(3):
        aux = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        out = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
        _lib.set_gemm_impl(26)
        try:
            gemm(a, b, bias=bias, act=2, aux_out=aux, out=out, aux_deriv=deriv)
            ran = _lib.gemm_last_kernel()
        finally:
            _lib.set_gemm_impl(-1)
        torch.cuda.synchronize()
        for name, t in (("C", out), ("aux", aux)):
            bad = ~torch.isfinite(t.float())
            if bad.any():
                rows = bad.any(1).nonzero().flatten()
                cols = bad.any(0).nonzero().flatten()
                print(f"deriv={deriv} trial={trial} kernel={ran} {name}: {int(bad.sum())} non-finite, rows "
                      f"{rows.min().item()}..{rows.max().item()} ({rows.numel()}), cols {cols.min().item()}.."
                      f"{cols.max().item()} ({cols.numel()}), tiles {sorted(set((r // 256, c // 256) for r, c in bad.nonzero().tolist()))[:12]}")
            else:
                print(f"deriv={deriv} trial={trial} kernel={ran} {name}: all finite")
