#!/usr/bin/env python3
"""fp8 (e4m3) forward GEMM tile sweep on the Transformer-big forward shapes
(8192 tokens), against the in-tree bf16 GEMM on the same shapes. One JSON line
per shape: us per tile config, the bf16 time, PF/s of the best fp8 config.

  python scripts/fp8_gemm_sweep.py --cfgs 3,4,6,7,8
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import fp8  # noqa: E402
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) for a, b in ev)
    return t[len(t) // 2] * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfgs", default="3,4,6,7,8")
    ap.add_argument("--tokens", type=int, default=8192)
    args = ap.parse_args()
    cfgs = [int(c) for c in args.cfgs.split(",") if c]
    T, d, ff = args.tokens, 1024, 4096
    shapes = [("qkv", T, 3 * d, d, False), ("o", T, d, d, False), ("ffn1", T, ff, d, True),
              ("ffn2", T, d, ff, False), ("xkv6", T, 12 * d, d, False), ("q", T, d, d, False)]
    dev = "cuda"
    torch.manual_seed(0)
    meta = fp8.Fp8Meta(dev)
    ia, ib = meta.slot("a"), meta.slot("b")
    for name, M, N, K, relu in shapes:
        A = torch.randn(M, K, device=dev).bfloat16()
        W = (torch.randn(N, K, device=dev) * 0.05).bfloat16()
        bias = torch.randn(N, device=dev)
        meta.scale[ia] = 448.0 / A.float().abs().max()
        meta.scale[ib] = 448.0 / W.float().abs().max()
        a8, b8 = fp8.quantize(A, meta, ia), fp8.quantize(W, meta, ib)
        ref = torch.nn.functional.linear(A.float(), W.float(), bias)
        if relu:
            ref = ref.relu()
        row = {"name": name, "M": M, "N": N, "K": K}
        best = None
        for c in cfgs:
            try:
                y, _ = fp8.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=relu, cfg=c)
                torch.cuda.synchronize()
            except RuntimeError:
                continue
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            t = timeit(lambda: fp8.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=relu, cfg=c))
            row[f"cfg{c}"] = round(t, 2)
            row[f"err{c}"] = float(f"{err:.1e}")
            if best is None or t < best[1]:
                best = (c, t)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        e = kk.EPI_BIAS_RELU if relu else kk.EPI_BIAS
        row["bf16_us"] = round(timeit(lambda: kk.gemm(A, W, C, M, N, K, K, K, N, True, True, e, bias=bias)), 2)
        row["best"] = best[0]
        row["best_pfs"] = round(2.0 * M * N * K / best[1] / 1e9, 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
