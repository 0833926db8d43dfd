#!/usr/bin/env python3
"""Weight-gradient kernel lab: dW[M,N] (f32) = dY[K,M]^T X[K,N], K = tokens,
both operands token-major (TN). Per shape: the lock-step 256x256 kernel
(cfg 12, the ragged launch's main loop) against the pipelined loop at 2x4
waves (cfg 20) and at 2x2 waves = one wave per SIMD (cfg 23 NS4, 24 NS5).
Also NT/NN shapes of the forward / dgrad for the same configs.
Graph-replayed back-to-back timings on random data."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import graph_time  # noqa

CFGS = [int(c) for c in os.environ.get("CFGS", "12,20,23,24,25,26").split(",")]
T = int(os.environ.get("TOKENS", "8192"))
base = [(512, 512), (1536, 512), (512, 2048), (2048, 512), (6144, 512), (7040, 512)]
big = [(1024, 1024), (3072, 1024), (1024, 4096), (4096, 1024), (12288, 1024), (7040, 1024)]
torch.manual_seed(0)
# the model's whole ragged weight-gradient launch (Transformer-base / -big):
# every layer's problems, bias sums fused where the model fuses them
def ragged_set(d, ff, L=6, vocab=7010, vpad=7040):
    enc = [(d, d, False), (3 * d, d, True), (d, ff, False), (ff, d, True)]
    dec = [(d, d, False), (3 * d, d, True), (d, d, True), (d, d, False), (ff, d, True), (d, ff, False)]
    return enc * L + dec * L + [(2 * L * d, d, True), (vocab, d, True)]

for name, d, ff in (("base", 512, 2048), ("big", 1024, 4096)):
    spec = ragged_set(d, ff)
    # problems of equal shape adjacent (as WgradQueue groups them)
    spec = sorted(spec, key=lambda s: (s[0], s[1]))
    dys, xs, dws, bs = [], [], [], []
    flops = 0
    for (n_out, n_in, bias) in spec:
        ld = 7040 if n_out == 7010 else n_out
        dy = (torch.rand(T, ld, device="cuda") * 2 - 1).bfloat16()
        dys.append(dy[:, :n_out] if ld != n_out else dy)
        xs.append((torch.rand(T, n_in, device="cuda") * 2 - 1).bfloat16())
        dws.append(torch.zeros(n_out, n_in, device="cuda"))
        bs.append(torch.zeros(n_out, device="cuda") if bias else None)
        flops += 2.0 * n_out * n_in * T
    row = []
    for impl in (0, 1, 2):
        kk.WGRAD_IMPL = impl

        def run():
            for c0 in range(0, len(spec), 64):
                kk.wgrad_ragged(dys[c0:c0 + 64], xs[c0:c0 + 64], dws[c0:c0 + 64], 0.0, bs[c0:c0 + 64])
        t = graph_time(run, n=5)
        row.append(f"impl{impl}={t:8.1f}us {flops/t/1e9:5.2f}PF")
    print(f"ragged {name} ({len(spec)} problems): " + "  ".join(row), flush=True)
kk.WGRAD_IMPL = 0

for name, shapes in (("base", base), ("big", big)):
    for M, N in shapes:
        dy = (torch.rand(T, M, device="cuda") * 2 - 1).bfloat16()
        x = (torch.rand(T, N, device="cuda") * 2 - 1).bfloat16()
        ref = None
        row = []
        for c in CFGS:
            C = torch.zeros(M, N, device="cuda", dtype=torch.float32)
            kk.gemm(dy, x, C, M, N, T, M, N, N, False, False, cfg=(c, 1))
            if ref is None:
                ref = dy.float().t() @ x.float()
            err = ((C - ref).abs().max() / ref.abs().max()).item()
            t = graph_time(lambda: kk.gemm(dy, x, C, M, N, T, M, N, N, False, False, cfg=(c, 1)))
            row.append(f"c{c}={t:7.1f}us {2*M*N*T/t/1e9:5.2f}PF{'' if err < 1e-3 else ' ERR%.1e' % err}")
        print(f"wgrad {name} {M}x{N}x{T}: " + "  ".join(row), flush=True)
# forward NT and dgrad NN at the model's shapes
for (M, N, K) in [(8192, 2048, 512), (8192, 1536, 512), (8192, 512, 2048), (8192, 7040, 512),
                  (8192, 4096, 1024), (8192, 3072, 1024), (8192, 1024, 4096), (8192, 12288, 1024)]:
    A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
    Bt = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
    Bn = (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    for kind, B, bkc, ldb in (("NT", Bt, True, K), ("NN", Bn, False, N)):
        row = []
        for c in [0, 4, 12] + CFGS[1:]:
            try:
                t = graph_time(lambda: kk.gemm(A, B, C, M, N, K, K, ldb, N, True, bkc, cfg=(c, 1)))
            except RuntimeError as e:
                row.append(f"c{c}=fail")
                continue
            row.append(f"c{c}={t:6.1f}us {2*M*N*K/t/1e9:5.2f}PF")
        print(f"{kind} {M}x{N}x{K}: " + "  ".join(row), flush=True)

