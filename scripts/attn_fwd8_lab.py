#!/usr/bin/env python3
"""e4m3 attention forward at the config-5 shape (B=16, H=16, L=512, hd=64),
non-causal, 10 calls -- a short program for rocprofv3 PMC
passes."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk

B, H, L, hd = 16, 16, 512, 64
sc = torch.full((1,), 8.0, device="cuda")
q8, k8, v8 = ((torch.randn(B, L, H, hd, device="cuda") * 8).to(torch.float8_e4m3fn) for _ in range(3))
kv = torch.full((B,), L, dtype=torch.int32, device="cuda")
for causal in (False,):
    for _ in range(10):
        kk.attn_fwd_fp8(q8, k8, v8, sc, sc, sc, kv, 0.125, causal)
torch.cuda.synchronize()
print("ok")
