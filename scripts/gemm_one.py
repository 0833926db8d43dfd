#!/usr/bin/env python3
"""Run one GEMM shape/config repeatedly (for rocprofv3 counter collection)."""
import argparse, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=8192)
ap.add_argument("--N", type=int, default=2048)
ap.add_argument("--K", type=int, default=512)
ap.add_argument("--kind", default="fwd")
ap.add_argument("--cfg", type=int, default=7)
ap.add_argument("--splits", type=int, default=1)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
M, N, K = a.M, a.N, a.K
if a.kind == "fwd":
    A = torch.randn(M, K, device="cuda").bfloat16(); B = torch.randn(N, K, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16); args = (A, B, C, M, N, K, K, K, N, True, True)
elif a.kind == "dgrad":
    A = torch.randn(M, K, device="cuda").bfloat16(); B = torch.randn(K, N, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16); args = (A, B, C, M, N, K, K, N, N, True, False)
else:
    A = torch.randn(K, M, device="cuda").bfloat16(); B = torch.randn(K, N, device="cuda").bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.float32); args = (A, B, C, M, N, K, M, N, N, False, False)
for _ in range(a.reps):
    kk.gemm(*args, cfg=(a.cfg, a.splits))
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(a.reps):
    kk.gemm(*args, cfg=(a.cfg, a.splits))
e.record(); torch.cuda.synchronize()
us = s.elapsed_time(e) / a.reps * 1e3
print(f"{a.kind} {M}x{N}x{K} cfg{a.cfg} s{a.splits}: {us:.2f} us  {2*M*N*K/us/1e6:.1f} TF")
