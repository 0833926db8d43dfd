#!/usr/bin/env python3
"""The Transformer-base (or -big) ragged weight-gradient launch alone, N
times, for counter collection (rocprofv3 --pmc ... -- python3 this).
The model's 62 problems (every layer's Dense weight gradients, bias sums
fused where the model fuses them), token-major operands of T tokens."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402

preset = os.environ.get("PRESET", "base")
reps = int(os.environ.get("REPS", "10"))
T = int(os.environ.get("TOKENS", "8192"))
d, ff = (512, 2048) if preset == "base" else (1024, 4096)
L = 6
enc = [(d, d, False), (3 * d, d, True), (d, ff, False), (ff, d, True)]
dec = [(d, d, False), (3 * d, d, True), (d, d, True), (d, d, False), (ff, d, True), (d, ff, False)]
spec = sorted(enc * L + dec * L + [(2 * L * d, d, True), (7010, d, True)], key=lambda s: (s[0], s[1]))
torch.manual_seed(0)
dys, xs, dws, bs = [], [], [], []
for n_out, n_in, bias in spec:
    ld = 7040 if n_out == 7010 else n_out
    dy = ((torch.rand(T, ld, device="cuda") * 2 - 1) * 0.1).bfloat16()
    dys.append(dy[:, :n_out] if ld != n_out else dy)
    xs.append((torch.rand(T, n_in, device="cuda") * 2 - 1).bfloat16())
    dws.append(torch.zeros(n_out, n_in, device="cuda"))
    bs.append(torch.zeros(n_out, device="cuda") if bias else None)
for _ in range(reps):
    kk.wgrad_ragged(dys, xs, dws, 0.0, bs)
torch.cuda.synchronize()
print("ok", len(spec), "problems")
