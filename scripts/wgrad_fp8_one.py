#!/usr/bin/env python3
"""Run the fp8 weight-gradient kernel (wgrad_fp8) and the bf16 ragged one on
the Transformer-big FFN problem set (T = 8192) repeatedly -- for rocprofv3
counter collection -- and print per-call times."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import fp8 as F
from tensorflow_distributed_on_gke_amd.ops import kernels as kk

T, reps = 8192, int(os.environ.get("REPS", "10"))
spec = [(4096, 1024)] * 6 + [(1024, 4096)] * 6
gm, am = F.Fp8Meta("cuda", fmt=1), F.Fp8Meta("cuda")
dys, xs, dws, sas, sbs, d16, x16 = [], [], [], [], [], [], []
for i, (M, N) in enumerate(spec):
    ga, ab = gm.slot(f"g{i}"), am.slot(f"x{i}")
    dys.append((torch.randn(T, M, device="cuda") * 4).to(F.BF8))
    xs.append((torch.randn(T, N, device="cuda") * 4).to(F.FP8))
    d16.append(torch.randn(T, M, device="cuda").bfloat16())
    x16.append(torch.randn(T, N, device="cuda").bfloat16())
    dws.append(torch.empty(M, N, device="cuda"))
    sas.append(gm.s(ga)), sbs.append(am.s(ab))
fl = sum(2.0 * M * N * T for M, N in spec)
for name, fn in (("fp8", lambda: F.wgrad_fp8(dys, sas, xs, sbs, dws, 0.0)),
                 ("bf16", lambda: kk.wgrad_ragged(d16, x16, dws, 0.0))):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) / reps * 1e3
    print(f"{name}: {us:.1f} us per call, {fl / us / 1e9:.2f} PF/s, {len(spec)} problems", flush=True)
