#!/usr/bin/env python3
"""hipBLASLt fp8 (torch._scaled_mm, per-tensor scales) vs the in-tree e4m3
GEMM (csrc/kernels/fp8.hip) on the Transformer-big seq-512 projection shapes."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import fp8 as F  # noqa: E402


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record(); b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


meta = F.Fp8Meta("cuda")
ia, ib = meta.slot("a"), meta.slot("b")
for M, N, K in [(8192, 3072, 1024), (8192, 1024, 4096), (8192, 4096, 1024), (8192, 12288, 1024)]:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    bias = torch.randn(N, device="cuda")
    a8 = F.quantize(a, meta, ia, record=False)
    w8 = F.quantize(w, meta, ib, record=False)
    ours = timeit(lambda: F.gemm_fp8(a8, w8, bias, meta, ia, ib))
    inv = torch.ones(1, device="cuda")
    try:
        y = torch._scaled_mm(a8, w8.t(), scale_a=inv, scale_b=inv, bias=bias.bfloat16(), out_dtype=torch.bfloat16)
        ref = F.gemm_fp8(a8, w8, bias, meta, ia, ib)[0]
        err = ((y.float() - ref.float()).abs().max() / ref.float().abs().max()).item()
        blas = timeit(lambda: torch._scaled_mm(a8, w8.t(), scale_a=inv, scale_b=inv, bias=bias.bfloat16(),
                                              out_dtype=torch.bfloat16))
        print(f"{M}x{N}x{K}: ours {ours:.1f} us  _scaled_mm {blas:.1f} us  (rel err {err:.2e})", flush=True)
    except Exception as e:  # noqa: BLE001
        print(f"{M}x{N}x{K}: ours {ours:.1f} us  _scaled_mm unavailable: {e}", flush=True)
