"""First step of a GPU job on a fresh box: import torch, touch the GPU, load the kernel library,
with timestamps (the first import on a fresh box pages the image in and can take minutes)."""
import os
import sys
import time

t = time.time()
import torch  # noqa: E402

print(f"import torch {time.time() - t:.1f}s", flush=True)
torch.zeros(1, device="cuda")
torch.cuda.synchronize()
print(f"gpu init {time.time() - t:.1f}s", flush=True)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_pytorch_cookbook_amd.ops import _lib  # noqa: E402

_lib.lib()
print(f"kernel library {time.time() - t:.1f}s loaded={_lib.is_loaded()}", flush=True)
