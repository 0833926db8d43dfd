#!/usr/bin/env python3
"""Fused projection + LayerNorm (gemm_ln) vs GEMM + ln_fwd on one shape,
repeated (timing, and a target for rocprofv3 counter collection)."""
import argparse, math, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk

ap = argparse.ArgumentParser()
ap.add_argument("--M", type=int, default=8192)
ap.add_argument("--K", type=int, default=512)
ap.add_argument("--reps", type=int, default=50)
a = ap.parse_args()
M, K, D = a.M, a.K, 512
dev = "cuda"
A = torch.randn(M, K, device=dev).bfloat16()
W = (torch.randn(D, K, device=dev) / math.sqrt(K)).bfloat16()
b = torch.randn(D, device=dev) * 0.1
x = torch.randn(M, D, device=dev).bfloat16()
g = torch.ones(D, device=dev)
be = torch.zeros(D, device=dev)
ctr = torch.zeros(1, dtype=torch.int64, device=dev)


def fused():
    kk.gemm_ln(A, W, b, x, g, be, 0.1, 1, ctr, 3)


def unfused():
    s = kk.linear_fwd(A, W, b)
    kk.ln_fwd(x, s, g, be, 0.1, 1, ctr, 3)


for name, fn in (("fused", fused), ("unfused", unfused)):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{name} M={M} K={K}: {s.elapsed_time(e) / a.reps * 1e3:.2f} us")
