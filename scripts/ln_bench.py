#!/usr/bin/env python3
"""LayerNorm forward/backward kernel timing at the Transformer-base shape
(8192 rows x 512): back-to-back launches timed with HIP events, with and
without dropout, plus the bytes each moves (effective bandwidth)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402

DEV = "cuda"


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    M = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    D = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    x = torch.randn(M, D, device=DEV).bfloat16()
    s = torch.randn(M, D, device=DEV).bfloat16()
    g = torch.rand(D, device=DEV) + 0.5
    b = torch.randn(D, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    dg = torch.zeros(D, device=DEV)
    db = torch.zeros(D, device=DEV)
    dbias = torch.zeros(D, device=DEV)
    out = {"M": M, "D": D}
    mb = M * D * 2 / 1e6
    for p in (0.0, 0.1):
        t = timeit(lambda: kk.ln_fwd(x, s, g, b, p, 1, ctr, 3))
        out[f"fwd_p{p}"] = round(t, 2)
        out[f"fwd_p{p}_GBs"] = round(4 * mb / t * 1e3, 0)
        y, h, mean, rstd = kk.ln_fwd(x, s, g, b, p, 1, ctr, 3)
        dy = torch.randn(M, D, device=DEV).bfloat16()
        t = timeit(lambda: kk.ln_bwd(dy, h, mean, rstd, g, dg, db, dbias, p, 1, ctr, 3))
        out[f"bwd_p{p}"] = round(t, 2)
        out[f"bwd_p{p}_GBs"] = round(4 * mb / t * 1e3, 0)
    t = timeit(lambda: kk.ln_fwd(x, s, g, b, 0.0, 1, ctr, 3, save=False))
    out["fwd_nosave"] = round(t, 2)
    z = torch.empty(M * D * 2, dtype=torch.bfloat16, device=DEV)
    out["copy_16MB_us"] = round(timeit(lambda: z[: M * D].copy_(z[M * D:])), 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
