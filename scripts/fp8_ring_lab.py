#!/usr/bin/env python3
"""Time the fp8 half-stage ring GEMM (cfg 10) against the 2-stage 128x128
(cfg 0) and 256x256 one-wave (cfg 9) kernels on the Transformer-big seq-512
shapes: e4m3 forward (bias + ReLU + e4m3 copy), e5m2 dgrad against the
transposed weight copy and against the plain weight (N-contiguous reads)."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
sys.path.insert(0, ROOT)
if os.environ.get("TDG_PKG_ROOT"):  # A/B against another built copy of the package
    sys.path.insert(0, os.path.abspath(os.environ["TDG_PKG_ROOT"]))
from tensorflow_distributed_on_gke_amd.ops import fp8 as F  # noqa: E402
from gemm_ceiling import graph_time  # noqa: E402

print("package:", os.path.dirname(F.__file__), flush=True)
torch.manual_seed(0)
meta, gm = F.Fp8Meta("cuda"), F.Fp8Meta("cuda", fmt=1)
ia, ib, io = meta.slot("a"), meta.slot("b"), meta.slot("o")
ig, igo = gm.slot("g"), gm.slot("go")
for (M, N, K) in [(8192, 4096, 1024), (8192, 1024, 4096), (8192, 3072, 1024), (8192, 1024, 1024),
                  (8192, 8192, 8192)]:
    a8 = (torch.randn(M, K, device="cuda") * 4).to(F.FP8)
    b8 = (torch.randn(N, K, device="cuda") * 4).to(F.FP8)
    bias = torch.randn(N, device="cuda")
    fl = 2.0 * M * N * K
    row = []
    ys = {}
    for c in (0, 9, 10):
        t = graph_time(lambda: F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=True, out8_slot=io, cfg=c))
        ys[c] = F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=True, out8_slot=io, cfg=c)[0].float()
        row.append(f"c{c}={t:7.1f}us {fl / t / 1e9:5.2f}PF")
    d = (ys[10] - ys[0]).abs().max().item()
    print(f"fwd {M}x{N}x{K}: " + "  ".join(row) + f"  |c10-c0|={d:.3g}", flush=True)
    g8 = (torch.randn(M, K, device="cuda") * 4).to(F.BF8)
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    row = []
    for c in (0, 9, 10):
        t = graph_time(lambda: F.gemm_bf8_dgrad(g8, gm, ig, b8, meta, ib, out, cfg=c))
        row.append(f"c{c}={t:7.1f}us {fl / t / 1e9:5.2f}PF")
    w8 = b8.t().contiguous()  # [K][N]: the plain weight of a dgrad producing N columns
    for c in (0, 10):
        t = graph_time(lambda: F.gemm_bf8_dgrad(g8, gm, ig, w8, meta, ib, out, cfg=c, w_plain=True))
        row.append(f"plain c{c}={t:7.1f}us {fl / t / 1e9:5.2f}PF")
    print(f"bwd {M}x{N}x{K}: " + "  ".join(row), flush=True)
