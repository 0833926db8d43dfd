#!/usr/bin/env python3
"""fp8 GEMM (plain, bf16 out, cfg 0 = 128x128 tiles, 2 workgroups per CU)
over K at fixed M x N: us per call and the per-tile-round fit
t = rounds * (F + nk * s) -- how much of a small-K tile round is fixed
(fill + epilogue) cost."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import fp8 as F
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import graph_time  # noqa

torch.manual_seed(0)
meta = F.Fp8Meta("cuda")
ia, ib = meta.slot("a"), meta.slot("b")
for M, N in ((8192, 4096), (8192, 1024), (8192, 3072)):
    rows = []
    for K in (256, 512, 1024, 2048, 4096, 8192):
        a8 = (torch.randn(M, K, device="cuda") * 4).to(F.FP8)
        b8 = (torch.randn(N, K, device="cuda") * 4).to(F.FP8)
        t = graph_time(lambda: F.gemm_fp8(a8, b8, None, meta, ia, ib, cfg=0))
        rows.append((K, t))
        print(f"{M}x{N}x{K}: {t:8.2f} us  {2.0 * M * N * K / t / 1e9:6.3f} PF/s", flush=True)
    tiles = (M // 128) * (N // 128)
    rounds = tiles / 512.0
    # least squares t / rounds = F + (K / 128) * s
    xs = [k / 128 for k, _ in rows]
    ys = [t / max(rounds, 1.0) for _, t in rows]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    s = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    f = my - s * mx
    print(f"  fit per tile round: F = {f:.2f} us fixed, s = {s:.3f} us per 128-deep K step "
          f"(K = 1024: fixed share {f / (f + 8 * s):.0%})", flush=True)
