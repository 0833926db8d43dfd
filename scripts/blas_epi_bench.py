#!/usr/bin/env python3
"""hipBLASLt (torch addmm / _addmm_activation: bias and bias+ReLU epilogues)
vs the in-tree GEMM (tuned tile) on the Transformer-base forward shapes."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for (M, N, K, relu) in [(8192, 1536, 512, False), (8192, 512, 512, False), (8192, 2048, 512, True),
                        (8192, 512, 2048, False), (8192, 7040, 512, False), (8192, 6144, 512, False)]:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / K ** 0.5).bfloat16()
    b = torch.randn(N, device="cuda")
    bb = b.bfloat16()
    ours = timeit(lambda: kk.linear_fwd(x, w, b, relu=relu))
    if relu:
        blas = timeit(lambda: torch._addmm_activation(bb, x, w.t(), use_gelu=False))
    else:
        blas = timeit(lambda: torch.addmm(bb, x, w.t()))
    print(f"{M}x{N}x{K} relu={relu}: ours {ours:.2f} us  hipBLASLt {blas:.2f} us", flush=True)
