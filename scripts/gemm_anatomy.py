#!/usr/bin/env python3
"""Where a one-tile-per-CU GEMM spends its time: the same launch timed at
several K (fixed cost = intercept, main loop = slope), next to a tiny kernel
(launch gap) and a fill of the output (store floor). 20 launches per HIP graph,
random operands."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk


def graph_time(fn, n=20, reps=7):
    fn(); torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay(); torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); g.replay(); b.record(); torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / n * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    torch.manual_seed(0)
    tiny = torch.zeros(64, device="cuda")
    print(f"tiny kernel (launch gap)      {graph_time(lambda: tiny.add_(1.0)):7.2f} us")
    for M, N in ((8192, 512), (8192, 2048)):
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        print(f"fill {M}x{N} bf16 ({C.numel() * 2 / 1e6:.0f} MB)   {graph_time(lambda: C.fill_(1.0)):7.2f} us")
    cases = [(8192, 512, (4, 13, 7, 0)), (8192, 2048, (12, 4, 7)), (8192, 1536, (12, 4, 7))]
    for M, N, cfgs in cases:
        for c in cfgs:
            row = []
            for K in (128, 256, 512, 1024, 2048, 4096):
                A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
                B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
                C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
                t = graph_time(lambda: kk.gemm(A, B, C, M, N, K, K, K, N, True, True, cfg=(c, 1)))
                row.append(f"K{K}:{t:6.2f}us/{2.0 * M * N * K / t / 1e6:5.0f}TF")
            print(f"{M}x{N} cfg{c:<2d} " + " ".join(row), flush=True)
        row = []
        for K in (128, 512, 2048):
            A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
            B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
            C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            t = graph_time(lambda: torch.mm(A, B.t(), out=C))
            row.append(f"K{K}:{t:6.2f}us/{2.0 * M * N * K / t / 1e6:5.0f}TF")
        print(f"{M}x{N} blt   " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
