#!/usr/bin/env python3
"""bf16 GEMM epilogue costs: the same NN dgrad / NT forward GEMM with the
plain, ReLU-backward (mask), beta-accumulate and bias(+ReLU) epilogues."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import graph_time  # noqa

torch.manual_seed(0)
for (M, N, K, cfgs) in [(8192, 2048, 512, (12,)), (8192, 4096, 1024, (12,)), (8192, 512, 2048, (13, 14)),
                        (8192, 512, 1536, (13, 14)), (8192, 1024, 4096, (22,))]:
    A = torch.randn(M, K, device="cuda").bfloat16()
    Bn = (torch.randn(K, N, device="cuda") * 0.05).bfloat16()
    Bt = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    C = torch.randn(M, N, device="cuda").bfloat16()
    aux = torch.randn(M, N, device="cuda").bfloat16()
    bias = torch.randn(N, device="cuda")
    fl = 2.0 * M * N * K
    for c in cfgs:
        rows = [
            ("NN plain", lambda: kk.gemm(A, Bn, C, M, N, K, K, N, N, True, False, cfg=(c, 1))),
            ("NN drelu", lambda: kk.gemm(A, Bn, C, M, N, K, K, N, N, True, False, kk.EPI_DRELU, aux=aux,
                                         ldaux=N, cfg=(c, 1))),
            ("NN beta1", lambda: kk.gemm(A, Bn, C, M, N, K, K, N, N, True, False, beta=1.0, cfg=(c, 1))),
            ("NT bias", lambda: kk.gemm(A, Bt, C, M, N, K, K, K, N, True, True, kk.EPI_BIAS, bias=bias,
                                        cfg=(c, 1))),
            ("NT bias+relu", lambda: kk.gemm(A, Bt, C, M, N, K, K, K, N, True, True, kk.EPI_BIAS_RELU,
                                             bias=bias, cfg=(c, 1))),
        ]
        out = []
        for name, fn in rows:
            try:
                t = graph_time(fn)
                out.append(f"{name} {t:6.1f}")
            except RuntimeError:
                out.append(f"{name} n/a")
        print(f"{M}x{N}x{K} c{c}: " + " | ".join(out), flush=True)
