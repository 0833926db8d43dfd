#!/usr/bin/env python3
"""A/B timing of the fp8 GEMM kernels (cfg 0 128x128 4-wave, cfg 9 256x256
one-wave, the fp8 weight-gradient kernel) on the Transformer-big seq-512
shapes. TDG_PKG_ROOT selects which copy of the package (and its built _C)
is imported, so two builds can be timed in one GPU call."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, os.environ.get("TDG_PKG_ROOT", ROOT))
from tensorflow_distributed_on_gke_amd.ops import fp8 as F  # noqa: E402
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402
from gemm_ceiling import graph_time  # noqa: E402

print("package:", os.path.dirname(F.__file__), flush=True)
torch.manual_seed(0)
meta, gm = F.Fp8Meta("cuda"), F.Fp8Meta("cuda", fmt=1)
ia, ib, io = meta.slot("a"), meta.slot("b"), meta.slot("o")
ig, igo = gm.slot("g"), gm.slot("go")
for (M, N, K) in [(8192, 4096, 1024), (8192, 1024, 4096), (8192, 3072, 1024), (8192, 8192, 8192)]:
    a8 = (torch.randn(M, K, device="cuda") * 4).to(F.FP8)
    b8 = (torch.randn(N, K, device="cuda") * 4).to(F.FP8)
    bias = torch.randn(N, device="cuda")
    fl = 2.0 * M * N * K
    row = []
    for c in (0, 9):
        t = graph_time(lambda: F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=True, out8_slot=io, cfg=c))
        row.append(f"c{c}={t:7.1f}us {fl / t / 1e9:5.2f}PF")
    print(f"fwd {M}x{N}x{K}: " + "  ".join(row), flush=True)
    g8 = (torch.randn(M, K, device="cuda") * 4).to(F.BF8)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    row = []
    for c in (0, 9):
        t = graph_time(lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, cfg=c))
        row.append(f"c{c}={t:7.1f}us {fl / t / 1e9:5.2f}PF")
    print(f"bwd {M}x{N}x{K}: " + "  ".join(row), flush=True)

T = 8192
spec = [(4096, 1024)] * 6 + [(1024, 4096)] * 6
dys, xs, dws, sas, sbs, d16, x16 = [], [], [], [], [], [], []
for i, (M, N) in enumerate(spec):
    dys.append((torch.randn(T, M, device="cuda") * 4).to(F.BF8))
    xs.append((torch.randn(T, N, device="cuda") * 4).to(F.FP8))
    d16.append(torch.randn(T, M, device="cuda").bfloat16())
    x16.append(torch.randn(T, N, device="cuda").bfloat16())
    dws.append(torch.empty(M, N, device="cuda"))
    sas.append(gm.s(gm.slot(f"g{i}"))), sbs.append(meta.s(meta.slot(f"x{i}")))
fl = sum(2.0 * M * N * T for M, N in spec)
t = graph_time(lambda: F.wgrad_fp8(dys, sas, xs, sbs, dws, 0.0))
print(f"wgrad fp8 12 FFN problems T={T}: {t:7.1f}us {fl / t / 1e9:5.2f}PF", flush=True)
t = graph_time(lambda: kk.wgrad_ragged(d16, x16, dws, 0.0))
print(f"wgrad bf16 12 FFN problems T={T}: {t:7.1f}us {fl / t / 1e9:5.2f}PF", flush=True)
