#!/usr/bin/env python3
"""GEMM microbenchmark on the Transformer-base training shapes: our MFMA kernel
(every tile config / split) vs torch.matmul (hipBLASLt) on the same random
bf16 operands. Interleaved timing in one process (HIP events, median of reps).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402

DEV = "cuda"


def timeit(fn, reps=30):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for _ in range(3):
        fn()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] * 1e3  # us


def shapes(tokens=8192, d=512, ff=2048, V=7010, Vp=7040):
    # (name, kind, M, N, K): fwd = x[M,K] W[N,K]^T ; dgrad = dy[M,N] W[N,K] ; wgrad = dy^T x
    return [
        ("qkv_fwd", "fwd", tokens, 3 * d, d),
        ("o_fwd", "fwd", tokens, d, d),
        ("ffn1_fwd", "fwd", tokens, ff, d),
        ("ffn2_fwd", "fwd", tokens, d, ff),
        ("vocab_fwd", "fwd", tokens, V, d),
        ("qkv_dgrad", "dgrad", tokens, d, 3 * d),
        ("o_dgrad", "dgrad", tokens, d, d),
        ("ffn1_dgrad", "dgrad", tokens, d, ff),
        ("ffn2_dgrad", "dgrad", tokens, ff, d),
        ("vocab_dgrad", "dgrad", tokens, d, Vp),
        ("qkv_wgrad", "wgrad", 3 * d, d, tokens),
        ("o_wgrad", "wgrad", d, d, tokens),
        ("ffn1_wgrad", "wgrad", ff, d, tokens),
        ("ffn2_wgrad", "wgrad", d, ff, tokens),
        ("vocab_wgrad", "wgrad", Vp, d, tokens),
    ]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=8192)
    ap.add_argument("--out", default="gpurun_out/gemm_bench.json")
    args = ap.parse_args()
    torch.manual_seed(0)
    res = []
    for name, kind, M, N, K in shapes(args.tokens):
        flops = 2.0 * M * N * K
        if kind == "fwd":
            A = torch.randn(M, K, device=DEV).bfloat16()
            B = torch.randn(N, K, device=DEV).bfloat16()
            C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ref = lambda: torch.matmul(A, B.t())  # noqa: E731
            args_ = (A, B, C, M, N, K, K, K, N, True, True)
            f32 = False
        elif kind == "dgrad":
            # dx[M, K'] = dy[M, Kc] W[Kc, K']  -> GEMM (M, N, K) with A=dy KC, B=W MC
            A = torch.randn(M, K, device=DEV).bfloat16()  # dy, contraction K
            B = torch.randn(K, N, device=DEV).bfloat16()  # W [K(out)][N(in)]
            C = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            ref = lambda: torch.matmul(A, B)  # noqa: E731
            args_ = (A, B, C, M, N, K, K, N, N, True, False)
            f32 = False
        else:
            # dW[M, N] = dy[K, M]^T x[K, N]
            A = torch.randn(K, M, device=DEV).bfloat16()
            B = torch.randn(K, N, device=DEV).bfloat16()
            C = torch.empty(M, N, device=DEV, dtype=torch.float32)
            ref = lambda: torch.matmul(A.t(), B)  # noqa: E731
            args_ = (A, B, C, M, N, K, M, N, N, False, False)
            f32 = True
        t_ref = timeit(ref)
        row = {"name": name, "M": M, "N": N, "K": K, "hipblaslt_us": round(t_ref, 2),
               "hipblaslt_tflops": round(flops / t_ref / 1e6, 1)}
        best = None
        for cfg in range(12):
            for splits in ((1, 2, 4, 8) if kind == "wgrad" else (1,)):
                if splits > 1 and K // splits < 256:
                    continue

                def run(cfg=cfg, splits=splits):
                    kk.gemm(*args_, cfg=(cfg, splits))

                t = timeit(run)
                key = f"cfg{cfg}_s{splits}"
                row[key] = round(t, 2)
                if best is None or t < best[1]:
                    best = (key, t)
        dflt = kk.choose_gemm(M, N, K, args_[-2], args_[-1])
        row["default"] = f"cfg{dflt[0]}_s{dflt[1]}"
        row["best"] = best[0]
        row["best_us"] = round(best[1], 2)
        row["best_tflops"] = round(flops / best[1] / 1e6, 1)
        # correctness spot check against hipBLASLt
        kk.gemm(*args_, cfg=dflt)
        r = ref().float()
        err = (C.float() - r).abs().max().item() / (r.abs().max().item() + 1e-6)
        row["rel_err"] = float(f"{err:.2e}")
        res.append(row)
        print(json.dumps(row), flush=True)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
