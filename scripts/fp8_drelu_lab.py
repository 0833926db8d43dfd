#!/usr/bin/env python3
"""The fp8 ReLU-backward dgrad (8192 x 4096 x 1024, e5m2 x e4m3) by epilogue
variant: bf16 output or not, bf16 or e4m3 mask, fused column sums or not --
against the same GEMM with the forward's bias + ReLU epilogue."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import fp8 as F
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import graph_time  # noqa

torch.manual_seed(0)
M, N, K = 8192, 4096, 1024
meta, gm = F.Fp8Meta("cuda"), F.Fp8Meta("cuda", fmt=1)
ia, ib, io, ih = meta.slot("a"), meta.slot("b"), meta.slot("o"), meta.slot("h")
ig, igo = gm.slot("g"), gm.slot("go")
a8 = (torch.randn(M, K, device="cuda") * 4).to(F.FP8)
b8 = (torch.randn(N, K, device="cuda") * 4).to(F.FP8)
g8 = (torch.randn(M, K, device="cuda") * 4).to(F.BF8)
bias = torch.randn(N, device="cuda")
aux = torch.randn(M, N, device="cuda").bfloat16()
aux8 = torch.relu(torch.randn(M, N, device="cuda")).to(F.FP8)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
cs = torch.zeros(N, device="cuda")
fl = 2.0 * M * N * K
rows = [
    ("fwd relu +C +h8", lambda: F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=True, out8_slot=io, cfg=0)),
    ("fwd relu h8 only", lambda: F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=True, out8_slot=io, cfg=0, want_y=False)),
    ("fwd plain +C", lambda: F.gemm_fp8(a8, b8, None, meta, ia, ib, cfg=0)),
    ("bwd +C aux16 +o8", lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, relu_aux=aux, out8_slot=igo, cfg=0)),
    ("bwd +C aux8 +o8", lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, relu_aux8=aux8, out8_slot=igo, cfg=0)),
    ("bwd aux8 +o8", lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, None, relu_aux8=aux8, out8_slot=igo, cfg=0)),
    ("bwd aux8 +o8 +colsum", lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, None, relu_aux8=aux8, out8_slot=igo,
                                                      colsum_out=cs)),
    ("bwd +C plain", lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, cfg=0)),
    ("bwd +C +o8", lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, out8_slot=igo, cfg=0)),
    ("bwd +C aux16", lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, relu_aux=aux, cfg=0)),
    ("bwd +C aux8", lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, relu_aux8=aux8, cfg=0)),
]
for r in range(2):
    for name, fn in rows:
        t = graph_time(fn)
        print(f"round {r} {name:24s} {t:7.1f} us  {fl / t / 1e9:5.2f} PF/s", flush=True)
