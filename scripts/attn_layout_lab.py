#!/usr/bin/env python3
"""Short-sequence attention (Transformer-base: B 64, H 8, L 128, hd 64) with
Q / K / V as separate contiguous tensors vs as views of the fused QKV GEMM
output [B, L, 3, H, hd] (the step's layout) -- forward and fused backward,
graph-replayed, us per call."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from attn_bench import graph_time  # noqa

B, H, L, hd = 64, 8, 128, 64
torch.manual_seed(0)
kv = torch.full((B,), L, dtype=torch.int32, device="cuda")
qkv = torch.randn(B, L, 3, H, hd, device="cuda").bfloat16()
sep = [qkv[:, :, i].contiguous() for i in range(3)]
fused = [qkv[:, :, i] for i in range(3)]
do = torch.randn(B, L, H, hd, device="cuda").bfloat16()
for causal in (False, True):
    for name, (q, k, v) in (("separate", sep), ("fused-view", fused)):
        o, lse = kk.attn_fwd(q, k, v, kv, 0.125, causal)
        dq, dk, dv = torch.empty_like(sep[0]), torch.empty_like(sep[0]), torch.empty_like(sep[0])
        tf = graph_time(lambda: kk.attn_fwd(q, k, v, kv, 0.125, causal))
        tb = graph_time(lambda: kk.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, kv, 0.125, causal))
        print(f"causal={causal} {name:10s}: fwd {tf:6.2f} us  bwd {tb:6.2f} us", flush=True)
