#!/usr/bin/env python3
"""GEMM structure ceiling: every tile config on large cubes and on the
model's fwd shapes, timed as 20 back-to-back launches inside a HIP graph
(what the training step sees), vs hipBLASLt (torch.mm)."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk

def graph_time(fn, n=20, reps=5):
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
    cfgs = [int(c) for c in os.environ.get("CFGS", "0,1,2,3,4,5,6,7,8,9,10,11").split(",")]
    shapes = [(8192, 8192, 8192), (4096, 4096, 4096), (8192, 2048, 512), (8192, 512, 2048), (8192, 1536, 512), (8192, 512, 512)]
    torch.manual_seed(0)
    for M, N, K in shapes:
        A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        fl = 2.0 * M * N * K
        row = []
        t = graph_time(lambda: torch.mm(A, B.t(), out=C))
        row.append(f"blt {t:8.2f}us {fl / t / 1e6:6.0f}TF")
        for c in cfgs:
            try:
                t = graph_time(lambda: kk.gemm(A, B, C, M, N, K, K, K, N, True, True, cfg=(c, 1)))
                row.append(f"c{c} {fl / t / 1e6:5.0f}")
            except RuntimeError:
                row.append(f"c{c}   n/a")
        print(f"{M}x{N}x{K}: " + " | ".join(row), flush=True)


if __name__ == "__main__":
    main()
