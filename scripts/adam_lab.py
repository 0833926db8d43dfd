#!/usr/bin/env python3
"""Adam kernel in isolation at the Transformer-base / -big parameter counts:
time per call and effective bandwidth (30 B / parameter: p, g, m, v read;
p, m, v written; bf16 shadow written), graph-replayed."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import kernels as kk
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gemm_ceiling import graph_time  # noqa

from tensorflow_distributed_on_gke_amd.ops._ext import C as _C
for var in (0, 1, 2, 3, 4):
  _C().adam_variant(var)
  print(f"variant {var}", flush=True)
  for n in (55_299_456, 198_672_256):
      p, g, m, v = (torch.randn(n, device="cuda") for _ in range(4))
      sh = torch.empty(n, device="cuda", dtype=torch.bfloat16)
      step = torch.zeros(1, dtype=torch.int64, device="cuda")
      t = graph_time(lambda: kk.adam(p, g, m, v, sh, step, 0.9, 0.98, 1e-9, 0.0, 512.0, 4000.0,
                                     zero_grad=False, inc_step=False), n=5)
      # the same after an L2/MALL flush (a 512 MB write between calls)
      junk = torch.empty(512 * 2 ** 20 // 4, device="cuda")

      def cold():
          junk.fill_(1.0)
          kk.adam(p, g, m, v, sh, step, 0.9, 0.98, 1e-9, 0.0, 512.0, 4000.0, zero_grad=False, inc_step=False)
      tf = graph_time(lambda: junk.fill_(1.0), n=5)
      tc = graph_time(cold, n=5) - tf
      cp = graph_time(lambda: p.copy_(g), n=5)
      print(f"n={n/1e6:.1f}M: adam {t:.1f} us = {30 * n / t / 1e6:.2f} TB/s | after 512 MB flush {tc:.1f} us "
            f"= {30 * n / tc / 1e6:.2f} TB/s | f32 copy {cp:.1f} us = {8 * n / cp / 1e6:.2f} TB/s", flush=True)
      del p, g, m, v, sh, junk
      torch.cuda.empty_cache()
