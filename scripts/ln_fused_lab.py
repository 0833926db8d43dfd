#!/usr/bin/env python3
"""Where the fused post-LN GEMM epilogues spend their time (tdg_gemm_ln.h):
each fused launch timed against the unfused pair it replaces (GEMM, then
ln_fwd / ln_bwd) and against itself with parts of the epilogue switched off
(kernels.LN_ABLATE bits: 1 dropout mask, 2 band exchange, 4 h / ds store,
8 row reductions, 16 y / dh store). Transformer-base shapes, back-to-back
launches, HIP-event timing (median of rounds).

    python scripts/ln_fused_lab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402

DEV = "cuda"
D, M = 512, 8192


def timeit(fn, reps=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    best = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        best.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(best)[len(best) // 2]


def main():
    torch.manual_seed(0)
    ctr = torch.tensor([1], dtype=torch.int64, device=DEV)
    p = 0.1
    g = torch.ones(D, device=DEV)
    b0 = torch.zeros(D, device=DEV)
    x = torch.randn(M, D, device=DEV).bfloat16()
    for K in (512, 2048):
        a = torch.randn(M, K, device=DEV).bfloat16()
        w = (torch.randn(D, K, device=DEV) * K ** -0.5).bfloat16()
        bias = torch.zeros(D, device=DEV)
        st = 3
        t_gemm = timeit(lambda: kk.linear_fwd(a, w, bias))
        s = kk.linear_fwd(a, w, bias)
        t_ln = timeit(lambda: kk.ln_fwd(x, s, g, b0, p, 5, ctr, 3))
        kbf = torch.zeros(M, D // 8, dtype=torch.uint8, device=DEV)
        t_lnk = timeit(lambda: kk.ln_fwd(x, s, g, b0, p, 5, ctr, 3, kbits=kbf))
        row = [f"fwd K={K}: gemm {t_gemm:6.1f}  ln_fwd {t_ln:6.1f} (kbits {t_lnk:6.1f})  sum {t_gemm + t_ln:6.1f} |"]
        for ab in (0, 1, 2, 4, 8, 16, 31):
            kk.LN_ABLATE = ab
            t = timeit(lambda: kk.linear_ln_fwd(a, w, bias, x, g, b0, p, 5, ctr, 3, stages=st))
            row.append(f" ab{ab}={t:6.1f}")
        kk.LN_ABLATE = 0
        print("".join(row), flush=True)
    for K, with_c in ((512, True), (1536, True), (2048, True)):
        dY = (torch.randn(M, K, device=DEV) * 0.1).bfloat16()
        w = (torch.randn(K, D, device=DEV) * K ** -0.5).bfloat16()
        c = (torch.randn(M, D, device=DEV) * 0.1).bfloat16()
        h = torch.randn(M, D, device=DEV).bfloat16()
        mean = h.float().mean(-1)
        rstd = torch.rsqrt(h.float().var(-1, unbiased=False) + 1e-6)
        outs = [torch.zeros(D, device=DEV) for _ in range(3)]
        st = 3 if K <= 512 else 4
        cc = c.clone()
        t_gemm = timeit(lambda: kk.linear_dgrad(dY, w, K, out=cc, beta=1.0))
        dy = kk.linear_dgrad(dY, w, K, out=c.clone(), beta=1.0)
        t_ln = timeit(lambda: kk.ln_bwd(dy, h, mean, rstd, g, *outs, p, 5, ctr, 3, defer=[]))
        kb = torch.zeros(M, D // 8, dtype=torch.uint8, device=DEV)
        t_lnk = timeit(lambda: kk.ln_bwd(dy, h, mean, rstd, g, *outs, p, 5, ctr, 3, defer=[], kbits=kb))
        row = [f"bwd K={K}: gemm {t_gemm:6.1f}  ln_bwd {t_ln:6.1f} (kbits {t_lnk:6.1f})  sum {t_gemm + t_ln:6.1f} |"]
        for ab in (0, 1, 2, 4, 8, 16, 31):
            kk.LN_ABLATE = ab
            t = timeit(lambda: kk.dgrad_ln_bwd(dY, w, c, h, mean, rstd, g, *outs, p, 5, ctr, 3, [],
                                               stages=st))
            row.append(f" ab{ab}={t:6.1f}")
        kk.LN_ABLATE = 0
        t = timeit(lambda: kk.dgrad_ln_bwd(dY, w, c, h, mean, rstd, g, *outs, p, 5, ctr, 3, [],
                                           stages=st, kbits=kb))
        row.append(f" kbits={t:6.1f}")
        print("".join(row), flush=True)
    torch.cuda.synchronize()
    kk.ln_xch_check()


if __name__ == "__main__":
    main()
