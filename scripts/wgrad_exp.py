#!/usr/bin/env python3
"""Weight-gradient GEMM experiment: dW[M,N] = dY^T X with K = tokens.
TN (as stored: both operands token-major, transposing LDS reads) vs NT on
pre-transposed operands (both K-contiguous), every config / split."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import graph_time  # noqa

shapes = [(512, 512, 8192), (2048, 512, 8192), (512, 2048, 8192), (1536, 512, 8192)]
for M, N, K in shapes:
    dy = torch.randn(K, M, device="cuda").bfloat16()
    x = torch.randn(K, N, device="cuda").bfloat16()
    dyt, xt = dy.t().contiguous(), x.t().contiguous()
    C = torch.empty(M, N, device="cuda", dtype=torch.float32)
    fl = 2.0 * M * N * K
    res = []
    for c in (0, 2, 4, 5, 6, 7, 8, 9, 10, 11, 1, 3):
        for sp in (1, 2, 4, 8):
            try:
                t_tn = graph_time(lambda: kk.gemm(dy, x, C, M, N, K, M, N, N, False, False, cfg=(c, sp)))
                t_nt = graph_time(lambda: kk.gemm(dyt, xt, C, M, N, K, K, K, N, True, True, cfg=(c, sp)))
                res.append((t_tn, t_nt, c, sp))
            except RuntimeError:
                pass
    best_tn = min(res, key=lambda r: r[0])
    best_nt = min(res, key=lambda r: r[1])
    tt = graph_time(lambda: (dy.t().contiguous(), x.t().contiguous()))
    print(f"{M}x{N}x{K}: TN best {best_tn[0]:.1f}us (c{best_tn[2]} s{best_tn[3]}, {fl/best_tn[0]/1e6:.0f} TF) | "
          f"NT best {best_nt[1]:.1f}us (c{best_nt[2]} s{best_nt[3]}, {fl/best_nt[1]/1e6:.0f} TF) | torch transposes {tt:.1f}us", flush=True)
    top = sorted(res)[:6]
    print("   TN top:", ", ".join(f"c{c}s{sp}={t:.1f}" for t, _, c, sp in top), flush=True)
