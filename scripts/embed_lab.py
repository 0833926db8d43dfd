#!/usr/bin/env python3
"""Embedding backward timing at the headline shape (8192 tokens, vocab 7040,
d 512, int64 ids): the deterministic path TDG_EMBED_GATHER selects (gather
or fixed-point atomics), HIP events, median of rounds."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402


def timeit(fn, reps=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    return sorted(ts)[len(ts) // 2]


M, V, D = 8192, 7040, 512
tok = torch.randint(4, V, (64, 128), device="cuda")
tok[:, 0], tok[:, -1] = 2, 3  # START / END of every sequence (the bench data's skew)
dout = torch.randn(64, 128, D, device="cuda").bfloat16()
dt = torch.zeros(V, D, device="cuda")
ctr = torch.tensor([3], dtype=torch.int64, device="cuda")
for p in (0.0, 0.1):
    t = timeit(lambda: kk.embed_bwd(tok, dout, dt, 22.6, p, 7, ctr, 2))
    print(f"gather={os.environ.get('TDG_EMBED_GATHER', '1')} p={p}: {t:.1f} us", flush=True)
