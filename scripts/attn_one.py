#!/usr/bin/env python3
"""Run the attention fwd+bwd repeatedly (for PMC collection): the base shape,
or ATTN_B / ATTN_H / ATTN_L (e.g. 16 / 16 / 512)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk
B = int(os.environ.get("ATTN_B", "64"))
H = int(os.environ.get("ATTN_H", "8"))
L = int(os.environ.get("ATTN_L", "128"))
hd = 64
q, k, v, do = (torch.randn(B, L, H, hd, device="cuda").bfloat16() for _ in range(4))
kv = torch.full((B,), L, dtype=torch.int32, device="cuda")
for _ in range(20):
    o, lse = kk.attn_fwd(q, k, v, kv, 0.125, False)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    kk.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, kv, 0.125, False)
torch.cuda.synchronize()
