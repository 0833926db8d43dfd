#!/usr/bin/env python3
"""In-tree MFMA GEMMs vs hipBLASLt (torch) on the exact forward / dgrad GEMMs
the Transformer-base and -big training steps issue (bias / bias+ReLU
epilogues, ReLU-backward dgrad), interleaved in one process on the same
random bf16 operands. Prints one JSON line per shape: hipBLASLt us, every
in-tree candidate's us, the best, and the max relative error vs hipBLASLt.

  python scripts/gemm_vs_blas.py --preset base --cfgs 0,4,7,13,14,12
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402


def timeit(fn, reps=20):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for _ in range(3):
        fn()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] * 1e3


def shapes(preset, T=8192):
    d, ff = (512, 2048) if preset == "base" else (1024, 4096)
    V = 7040
    fwd = [("qkv", T, 3 * d, d, "bias"), ("o", T, d, d, "bias"), ("ffn1", T, ff, d, "relu"),
           ("ffn2", T, d, ff, "bias"), ("vocab", T, V, d, "bias"), ("xkv6", T, 12 * d, d, "bias")]
    dgr = [("qkv", T, d, 3 * d, None), ("o", T, d, d, None), ("ffn1", T, d, ff, None),
           ("ffn2", T, ff, d, "drelu"), ("vocab", T, d, V, None), ("xkv6", T, d, 12 * d, None)]
    return [("fwd",) + s for s in fwd] + [("dgrad",) + s for s in dgr]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="base")
    ap.add_argument("--cfgs", default="0,4,7,13,14,12")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    cfgs = [int(c) for c in args.cfgs.split(",") if c]
    torch.manual_seed(0)
    dev = "cuda"
    tot = {"blas": 0.0, "best": 0.0}
    for kind, name, M, N, K, epi in shapes(args.preset):
        if args.only and name not in args.only.split(","):
            continue
        fl = 2.0 * M * N * K
        A = torch.randn(M, K, device=dev).bfloat16()
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if kind == "fwd":
            W = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
            b = torch.randn(N, device=dev)
            b16 = b.bfloat16()
            e = kk.EPI_BIAS_RELU if epi == "relu" else kk.EPI_BIAS
            if epi == "relu":
                ref = lambda: torch._addmm_activation(b16, A, W.t(), use_gelu=False, out=C)  # noqa: E731
            else:
                ref = lambda: torch.addmm(b16, A, W.t(), out=C)  # noqa: E731

            def mine(cfg):
                kk.gemm(A, W, C, M, N, K, K, K, N, True, True, e, bias=b, cfg=cfg)
        else:
            W = (torch.randn(K, N, device=dev) * 0.05).bfloat16()  # [out=K][in=N]
            aux = torch.randn(M, N, device=dev).bfloat16() if epi == "drelu" else None
            if aux is not None:
                ref = lambda: torch.mul(torch.mm(A, W), aux > 0, out=C)  # noqa: E731
            else:
                ref = lambda: torch.mm(A, W, out=C)  # noqa: E731

            def mine(cfg):
                kk.gemm(A, W, C, M, N, K, K, N, N, True, False,
                        kk.EPI_DRELU if aux is not None else kk.EPI_NONE, aux=aux,
                        ldaux=N if aux is not None else 0, cfg=cfg)
        ref()
        r = C.float().clone()
        row = {"kind": kind, "name": name, "M": M, "N": N, "K": K, "epi": epi}
        row["blas_us"] = round(timeit(ref), 2)
        best = None
        for c in cfgs:
            try:
                mine((c, 1))
                torch.cuda.synchronize()
            except RuntimeError:
                continue
            err = ((C.float() - r).abs().max() / (r.abs().max() + 1e-6)).item()
            t = timeit(lambda: mine((c, 1)))
            row[f"cfg{c}"] = round(t, 2)
            row[f"err{c}"] = float(f"{err:.1e}")
            if best is None or t < best[1]:
                best = (c, t)
        row["best"] = best[0]
        row["best_us"] = round(best[1], 2)
        row["best_tf"] = round(fl / best[1] / 1e6, 1)
        row["blas_tf"] = round(fl / row["blas_us"] / 1e6, 1)
        tot["blas"] += row["blas_us"]
        tot["best"] += row["best_us"]
        print(json.dumps(row), flush=True)
    print(json.dumps({"total_us": tot}), flush=True)


if __name__ == "__main__":
    main()
