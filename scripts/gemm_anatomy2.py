#!/usr/bin/env python3
"""Fixed cost of a one-tile-per-CU GEMM: output row pitch (power-of-two vs
padded) and tile count (M), random operands, 20 launches per HIP graph."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk
from gemm_anatomy import graph_time


def main():
    torch.manual_seed(0)
    for N, cfg in ((2048, 12), (512, 7)):
        for M in (8192, 4096, 2048):
            for K in (128, 512):
                A = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
                B = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16()
                row = []
                for pad in (0, 8, 64, 256):
                    ldc = N + pad
                    C = torch.empty(M, ldc, device="cuda", dtype=torch.bfloat16)
                    t = graph_time(lambda: kk.gemm(A, B, C, M, N, K, K, K, ldc, True, True, cfg=(cfg, 1)))
                    row.append(f"ldc+{pad}:{t:6.2f}us")
                Cs = torch.empty(M, N + 64, device="cuda", dtype=torch.bfloat16)
                tf = graph_time(lambda: Cs[:, :N].fill_(1.0))
                print(f"{M}x{N}x{K} cfg{cfg}: " + " ".join(row) + f"  | strided fill {tf:6.2f}us", flush=True)


if __name__ == "__main__":
    main()
