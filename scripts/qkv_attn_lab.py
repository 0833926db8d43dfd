"""Per-call time (HIP events, back to back) of the fused Q|K|V projection +
attention forward against the projection GEMM + attention forward it
replaces, at the Transformer-base / big self-attention shapes."""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402


def t(fn, n=50):
    for _ in range(5):
        fn()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(n):
        fn()
    e[1].record()
    e[1].synchronize()
    return e[0].elapsed_time(e[1]) / n * 1000.0


dev = "cuda"
for B, L, H, causal in [(64, 128, 8, False), (64, 128, 8, True), (64, 128, 16, False)]:
    d = 64 * H
    x = torch.randn(B * L, d, device=dev).bfloat16()
    w = (torch.randn(3 * d, d, device=dev) / math.sqrt(d)).bfloat16()
    b = torch.randn(3 * d, device=dev) * 0.1
    kv = torch.randint(L // 2, L + 1, (B,), device=dev, dtype=torch.int32)

    def two():
        q5 = kk.linear_fwd(x, w, b).view(B, L, 3, H, 64)
        kk.attn_fwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], kv, 0.125, causal)

    def gemm_only():
        kk.linear_fwd(x, w, b)

    r = {"gemm": t(gemm_only), "gemm+attn": t(two)}
    r["fused"] = t(lambda: kk.qkv_attn_fwd(x, w, b, B, H, kv, 0.125, causal))
    print(f"B{B} L{L} H{H} causal={causal}: "
          + "  ".join(f"{k}={v:.2f}us" for k, v in r.items()), flush=True)

# backward: output-projection dgrad + attention backward vs the in-kernel dO
for B, L, H, causal in [(64, 128, 8, False), (64, 128, 8, True), (64, 128, 16, False)]:
    d = 64 * H
    q, k, v = (torch.randn(B, L, H, 64, device=dev).bfloat16() for _ in range(3))
    kv = torch.randint(L // 2, L + 1, (B,), device=dev, dtype=torch.int32)
    o, lse = kk.attn_fwd(q, k, v, kv, 0.125, causal)
    dy2 = (torch.randn(B * L, d, device=dev) * 0.1).bfloat16()
    wo = (torch.randn(d, d, device=dev) / math.sqrt(d)).bfloat16()
    dq, dk, dv = (torch.empty_like(x) for x in (q, k, v))

    def two():
        do = kk.linear_dgrad(dy2, wo, d)
        kk.attn_bwd(q, k, v, o, do.view(B, L, H, 64), lse, dq, dk, dv, kv, 0.125, causal)

    def attn_only():
        kk.attn_bwd(q, k, v, o, o, lse, dq, dk, dv, kv, 0.125, causal)

    r = {"attn_bwd": t(attn_only), "dgrad+attn_bwd": t(two),
         "fused": t(lambda: kk.attn_bwd_fdo(q, k, v, o, dy2, wo, lse, dq, dk, dv, kv, 0.125, causal))}
    print(f"bwd B{B} L{L} H{H} causal={causal}: " + "  ".join(f"{k_}={v_:.2f}us" for k_, v_ in r.items()),
          flush=True)

# cross-attention forward: Q projection + attention vs the fused form
for B, L, H in [(64, 128, 8), (64, 128, 16)]:
    d = 64 * H
    x = torch.randn(B * L, d, device=dev).bfloat16()
    w = (torch.randn(d, d, device=dev) / math.sqrt(d)).bfloat16()
    b = torch.randn(d, device=dev) * 0.1
    kv5 = torch.randn(B, L, 2, H, 64, device=dev).bfloat16()
    kv = torch.randint(L // 2, L + 1, (B,), device=dev, dtype=torch.int32)

    def two():
        q = kk.linear_fwd(x, w, b)
        kk.attn_fwd(q.view(B, L, H, 64), kv5[:, :, 0], kv5[:, :, 1], kv, 0.125, False)

    r = {"qproj+attn": t(two),
         "fused": t(lambda: kk.qkv_attn_fwd(x, w, b, B, H, kv, 0.125, False, k=kv5[:, :, 0], v=kv5[:, :, 1]))}
    print(f"cross B{B} L{L} H{H}: " + "  ".join(f"{k_}={v_:.2f}us" for k_, v_ in r.items()), flush=True)
