"""Dump the attention backward of one fixed GPT-2-small-shaped input (for bitwise A/B of kernel
variants chosen by DPC_ATTN_VAR in separate processes): python attn_dump.py OUT.pt"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from distributed_pytorch_cookbook_amd.ops.attention import attention_bwd, attention_fwd  # noqa: E402

torch.manual_seed(0)
N, S, H, hd = 8, 1023, 12, 64
qkv = torch.randn(N * S, 3 * H * hd, device="cuda").bfloat16()
o, lse = attention_fwd(qkv, N, S, H, hd)
do = torch.randn(N * S, H * hd, device="cuda").bfloat16()
dqkv = attention_bwd(do, qkv, o, lse, N, S, H, hd)
torch.save(dqkv.cpu(), sys.argv[1])
