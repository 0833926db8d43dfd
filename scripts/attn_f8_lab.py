#!/usr/bin/env python3
"""Timing of the fp8 attention backward (attention.hip attn_bwd_f8_kernel)
against the bf16 backward (dQ + dK/dV pipelined kernels) on config 5's
attention shape: B 16, H 16, L 512, hd 64 (HIP events, median of rounds).

    python scripts/attn_f8_lab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.ops import fp8 as F  # noqa: E402
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402

DEV = "cuda"


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


def main():
    B, H, L, hd = (int(os.environ.get(k, v)) for k, v in (("B", "16"), ("H", "16"), ("L", "512"), ("HD", "64")))
    torch.manual_seed(0)
    meta, gmeta = F.Fp8Meta(DEV), F.Fp8Meta(DEV, fmt=1)
    sq = meta.slot("q")
    ido, ids, ig = gmeta.slot("do"), gmeta.slot("ds"), gmeta.slot("g")
    meta.scale[sq] = 64.0
    gmeta.scale.fill_(2.0 ** 16)
    x = [torch.randn(B, L, H, hd, device=DEV).bfloat16() for _ in range(3)]
    x8 = [F.quantize(t, meta, sq, record=False).view(t.shape) for t in x]
    xq = [(t8.float() / 64.0).bfloat16() for t8 in x8]
    do = (torch.randn(B, L, H, hd, device=DEV) * 0.01).bfloat16()
    do8 = F.quantize(do, gmeta, ido, record=False).view(do.shape)
    for causal in (False, True):
        o, lse = kk.attn_fwd_fp8(x8[0], x8[1], x8[2], meta.s(sq), meta.s(sq), meta.s(sq), None,
                                 hd ** -0.5, causal)
        dq, dk, dv = (torch.empty_like(t) for t in xq)
        t_bf = timeit(lambda: kk.attn_bwd(xq[0], xq[1], xq[2], o, do, lse, dq, dk, dv, None,
                                          hd ** -0.5, causal))
        d8 = torch.empty(B, L, 3, H, hd, dtype=torch.float8_e5m2, device=DEV)
        part = torch.empty(B, 3 * H * hd, device=DEV)
        t_f8 = timeit(lambda: kk.attn_bwd_f8(
            x8[0], x8[1], x8[2], meta.s(sq), meta.s(sq), meta.s(sq), o, do8, gmeta.s(ido), lse, None,
            hd ** -0.5, causal, gmeta.s(ids), gmeta.a(ids), dq8=d8[:, :, 0], dk8=d8[:, :, 1],
            dv8=d8[:, :, 2], sg8=gmeta.s(ig), amaxg8=gmeta.a(ig), cs_part=part, cs_ld=3 * H * hd,
            cs_q=0, cs_k=H * hd, cs_v=2 * H * hd))
        fl = 5 * 2 * B * H * L * L * hd * (0.5 if causal else 1.0)
        print(f"B{B} H{H} L{L} causal={causal}: bf16 bwd {t_bf:7.1f} us   fp8 bwd {t_f8:7.1f} us "
              f"({fl / t_f8 / 1e6:.0f} TF/s on the 5 products)", flush=True)


if __name__ == "__main__":
    main()
