#!/usr/bin/env python3
"""fp8 GEMM lab: the 128x128 / 4-wave kernel (cfg 0), the other table
configs, and the 256x256 one-wave-per-SIMD kernel (cfg 9) on the
Transformer-big seq-512 shapes (forward e4m3 x e4m3, backward e5m2 x e4m3
with the ReLU-backward epilogue). Graph-replayed, random data."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import fp8 as F
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import graph_time  # noqa

torch.manual_seed(0)
meta, gm = F.Fp8Meta("cuda"), F.Fp8Meta("cuda", fmt=1)
ia, ib, io = meta.slot("a"), meta.slot("b"), meta.slot("o")
ig, igo = gm.slot("g"), gm.slot("go")
for (M, N, K) in [(8192, 4096, 1024), (8192, 1024, 4096), (8192, 3072, 1024), (8192, 12288, 1024),
                  (8192, 1024, 1024), (8192, 2048, 512), (8192, 8192, 8192)]:
    a8 = (torch.randn(M, K, device="cuda") * 4).to(F.FP8)
    b8 = (torch.randn(N, K, device="cuda") * 4).to(F.FP8)
    bias = torch.randn(N, device="cuda")
    fl = 2.0 * M * N * K
    row = []
    for c in (0, 3, 4, 8, 9):
        t = graph_time(lambda: F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=True, out8_slot=io, cfg=c))
        row.append(f"c{c}={t:7.1f}us {fl / t / 1e9:5.2f}PF")
    print(f"fwd {M}x{N}x{K}: " + "  ".join(row), flush=True)
    g8 = (torch.randn(M, K, device="cuda") * 4).to(F.BF8)
    aux = torch.randn(M, N, device="cuda").bfloat16()
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    row = []
    for c in (0, 9):
        t = graph_time(lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, relu_aux=aux,
                                                out8_slot=igo, cfg=c))
        row.append(f"c{c}={t:7.1f}us {fl / t / 1e9:5.2f}PF")
    print(f"bwd-drelu {M}x{N}x{K}: " + "  ".join(row), flush=True)
