#!/usr/bin/env python3
"""Interleaved timing of the 256x256 GEMM main loops, lock-step vs ping-pong
(TDG_GEMM256_PP), on the Transformer-base shapes and the model's ragged
weight-gradient launch, in ONE process (HIP events, median of rounds)."""
import statistics
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402
from tensorflow_distributed_on_gke_amd.ops._ext import C  # noqa: E402

DEV = "cuda"


def bf(*s):
    return (torch.rand(*s, device=DEV) * 2 - 1).to(torch.bfloat16)


def timeit(fn, reps=20):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1000.0


def main():
    M = 8192
    cases = {}
    for (N, K, epi) in [(1536, 512, kk.EPI_BIAS), (2048, 512, kk.EPI_BIAS_RELU), (6144, 512, kk.EPI_BIAS),
                        (7010, 512, kk.EPI_BIAS)]:
        x, w, b = bf(M, K), bf(N, K), torch.rand(N, device=DEV)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        cases[f"NT {M}x{N}x{K} epi{epi}"] = (
            lambda x=x, w=w, b=b, out=out, N=N, K=K, epi=epi:
            kk.gemm(x, w, out, M, N, K, K, K, N, True, True, epi, bias=b, cfg=(12, 1)), 2 * M * N * K)
    dy, w2, h = bf(M, 512), bf(512, 2048), bf(M, 2048)
    o2 = torch.empty(M, 2048, dtype=torch.bfloat16, device=DEV)
    cases["NN 8192x2048x512 drelu"] = (
        lambda: kk.gemm(dy, w2, o2, M, 2048, 512, 512, 2048, 2048, True, False, kk.EPI_DRELU, aux=h,
                        ldaux=2048, cfg=(12, 1)), 2 * M * 2048 * 512)
    # the base model's ragged weight-gradient launch (per layer shapes x 6 + vocab)
    spec = ([(1536, 512)] * 12 + [(512, 512)] * 24 + [(2048, 512)] * 12 + [(512, 2048)] * 12 +
            [(6144, 512), (7010, 512)])
    dys = [bf(M, -(-n // 64) * 64)[:, :n] for n, _ in spec]  # padded ld (vocab 7010 -> 7040)
    xs = [bf(M, k) for _, k in spec]
    dws = [torch.empty(n, k, dtype=torch.float32, device=DEV) for n, k in spec]
    flops = sum(2 * M * n * k for n, k in spec)
    cases[f"ragged wgrad ({len(spec)} problems)"] = (
        lambda: kk.wgrad_ragged(dys, xs, dws, beta=0.0), flops)
    res = {k: {0: [], 1: []} for k in cases}
    for rnd in range(5):
        for pp in (0, 1):
            C().set_gemm256_pp(bool(pp))
            for k, (fn, _) in cases.items():
                res[k][pp].append(timeit(fn, 10 if "ragged" in k else 30))
    print(f"{'case':40s} {'lockstep us':>12s} {'pingpong us':>12s} {'PF/s lk':>8s} {'PF/s pp':>8s}")
    for k, (fn, fl) in cases.items():
        a, b = statistics.median(res[k][0]), statistics.median(res[k][1])
        print(f"{k:40s} {a:12.2f} {b:12.2f} {fl / a / 1e9:8.3f} {fl / b / 1e9:8.3f}")


if __name__ == "__main__":
    main()
