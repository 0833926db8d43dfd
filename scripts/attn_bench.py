#!/usr/bin/env python3
"""Attention fwd / bwd timing, HIP-graph replay of 20 calls. Default shape:
Transformer-base (B=64, H=8, L=128, hd=64); ATTN_B / ATTN_H / ATTN_L set
another (the big seq-512 config: ATTN_B=16 ATTN_H=16 ATTN_L=512). Prints
us per call and PF/s (causal counts the unmasked half)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("TDG_PKG_ROOT"):  # A/B against another built copy of the package
    sys.path.insert(0, os.path.abspath(os.environ["TDG_PKG_ROOT"]))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk

def graph_time(fn, n=20):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); g.replay(); b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3

B = int(os.environ.get("ATTN_B", "64"))
H = int(os.environ.get("ATTN_H", "8"))
L = int(os.environ.get("ATTN_L", "128"))
hd = 64
for causal in ((False, True) if __name__ == "__main__" else ()):
    q, k, v, do = (torch.randn(B, L, H, hd, device="cuda").bfloat16() for _ in range(4))
    kv = torch.full((B,), L, dtype=torch.int32, device="cuda")
    o, lse = kk.attn_fwd(q, k, v, kv, 0.125, causal)
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    tf = graph_time(lambda: kk.attn_fwd(q, k, v, kv, 0.125, causal))
    tb = graph_time(lambda: kk.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, kv, 0.125, causal))
    fl = 4.0 * B * H * L * L * hd * (0.5 if causal else 1.0)
    if os.environ.get("ATTN_FP8") and kk.attn_fwd_fp8_ok(L, L, hd):
        sc = torch.full((1,), 8.0, device="cuda")
        q8, k8, v8 = ((x.float() * 8.0).to(torch.float8_e4m3fn) for x in (q, k, v))
        t8 = graph_time(lambda: kk.attn_fwd_fp8(q8, k8, v8, sc, sc, sc, kv, 0.125, causal))
        print(f"B={B} H={H} L={L} causal={causal}: e4m3 fwd {t8:.2f} us ({fl / t8 / 1e9:.3f} PF/s)", flush=True)
    print(f"B={B} H={H} L={L} causal={causal}: "
          f"fwd {tf:.2f} us ({fl / tf / 1e9:.3f} PF/s)  bwd {tb:.2f} us ({2.5 * fl / tb / 1e9:.3f} PF/s)",
          flush=True)
