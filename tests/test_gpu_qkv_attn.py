"""The fused self-attention input projection + attention forward
(attention.hip qkv_attn_fwd_kernel: one launch per layer for sequences of
<= 128 tokens) against the two-launch path it replaces -- the Q|K|V GEMM
(linear_fwd) then attn_fwd on its output -- and the attention against a plain
fp32 PyTorch softmax(Q K^T / sqrt(hd) + mask) V (reference:
transformer_model.py:73-166, MultiHeadAttention with the padding / look-ahead
masks)."""
import math

import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import kernels as kk

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(B, L, H, causal, lens, seed=0):
    d = 64 * H
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(B * L, d, generator=g)).to(torch.bfloat16).to(DEV)
    w = (torch.randn(3 * d, d, generator=g) / math.sqrt(d)).to(torch.bfloat16).to(DEV)
    b = (torch.randn(3 * d, generator=g) * 0.1).to(DEV)
    kv = torch.tensor(lens, dtype=torch.int32, device=DEV) if lens is not None else None
    return x, w, b, kv, d


@pytest.mark.parametrize("B,L,H,causal,pad", [
    (64, 128, 8, False, True), (64, 128, 8, True, True), (16, 100, 8, False, True),
    (8, 37, 8, True, False), (16, 128, 16, False, True), (4, 128, 8, False, False),
])
def test_qkv_attn_matches_two_launches(B, L, H, causal, pad):
    g = torch.Generator().manual_seed(B + L)
    lens = torch.randint(1, L + 1, (B,), generator=g).tolist() if pad else None
    if pad:
        lens[0] = 0  # an all-padding row: the reference's uniform softmax
    x, w, b, kv, d = _case(B, L, H, causal, lens)
    hd = 64
    scale = 1.0 / math.sqrt(hd)
    r = kk.qkv_attn_fwd(x, w, b, B, H, kv, scale, causal)
    assert r is not None
    qkv, o, lse = r
    qkv0 = kk.linear_fwd(x, w, b)
    q5 = qkv0.view(B, L, 3, H, hd)
    o0, lse0 = kk.attn_fwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], kv, scale, causal)
    torch.cuda.synchronize()
    assert torch.equal(qkv, qkv0), "projection output differs from the GEMM's"
    assert torch.equal(o, o0), f"O differs: {(o.float() - o0.float()).abs().max().item()}"
    assert torch.equal(lse, lse0)
    # fp32 reference of the attention on the (bf16) projection output
    qf, kf, vf = (q5[:, :, i].float().permute(0, 2, 1, 3) for i in range(3))
    s = qf @ kf.transpose(-1, -2) * scale
    mask = torch.zeros(B, 1, L, L, device=DEV)
    if kv is not None:
        mask = mask + (torch.arange(L, device=DEV)[None, None, None, :] >= kv[:, None, None, None]).float()
    if causal:
        mask = torch.maximum(mask, torch.triu(torch.ones(L, L, device=DEV), 1)[None, None])
    p = torch.softmax(s + mask * -1e9, dim=-1)
    ref = (p @ vf).permute(0, 2, 1, 3)
    err = (o.float() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-3, err


def test_qkv_attn_declines_long_sequences():
    x, w, b, kv, d = _case(2, 200, 8, False, None)
    assert kk.qkv_attn_fwd(x, w, b, 2, 8, None, 0.125, False) is None


@pytest.mark.parametrize("B,Lq,Lk,H,causal,pad", [
    (64, 128, 128, 8, False, True), (64, 128, 128, 8, True, True), (16, 100, 100, 8, False, True),
    (8, 37, 37, 8, True, False), (16, 128, 128, 16, False, True), (16, 127, 128, 8, False, True),
])
def test_attn_bwd_fdo_matches_two_launches(B, Lq, Lk, H, causal, pad):
    """The fused backward with the output-projection dgrad in-kernel
    (attn_bwd_fused_kernel FDO) against linear_dgrad + attn_bwd: bitwise."""
    d, hd = 64 * H, 64
    g = torch.Generator().manual_seed(B * Lq + H)
    mk = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc).to(torch.bfloat16).to(DEV)  # noqa: E731
    q, k, v = mk(B, Lq, H, hd), mk(B, Lk, H, hd), mk(B, Lk, H, hd)
    lens = torch.randint(1, Lk + 1, (B,), generator=g) if pad else None
    if pad:
        lens[0] = 0
    kv = lens.to(torch.int32).to(DEV) if pad else None
    scale = 1.0 / math.sqrt(hd)
    o, lse = kk.attn_fwd(q, k, v, kv, scale, causal and Lq == Lk)
    causal = causal and Lq == Lk
    dy2 = mk(B * Lq, d, sc=0.1)
    wo = mk(d, d, sc=1.0 / math.sqrt(d))
    outs = []
    for fused in (True, False):
        dq, dk, dv = (torch.empty_like(t) for t in (q, k, v))
        if fused:
            assert kk.attn_bwd_fdo(q, k, v, o, dy2, wo, lse, dq, dk, dv, kv, scale, causal)
        else:
            do = kk.linear_dgrad(dy2, wo, d)
            kk.attn_bwd(q, k, v, o, do.view(B, Lq, H, hd), lse, dq, dk, dv, kv, scale, causal)
        outs.append((dq, dk, dv))
    torch.cuda.synchronize()
    for a, b, n in zip(outs[0], outs[1], ("dq", "dk", "dv")):
        assert torch.equal(a, b), f"{n}: {(a.float() - b.float()).abs().max().item()}"


@pytest.mark.parametrize("B,T,S,H,pad", [(64, 128, 128, 8, True), (16, 100, 77, 8, True),
                                         (8, 37, 128, 16, False), (4, 128, 64, 8, True)])
def test_cross_q_attn_matches_two_launches(B, T, S, H, pad):
    """The cross-attention form of the fused forward (Q projection in-kernel,
    K / V from the batched K|V projection) against linear_fwd + attn_fwd."""
    d, hd = 64 * H, 64
    g = torch.Generator().manual_seed(B * T + S)
    x = torch.randn(B * T, d, generator=g).to(torch.bfloat16).to(DEV)
    w = (torch.randn(d, d, generator=g) / math.sqrt(d)).to(torch.bfloat16).to(DEV)
    b = (torch.randn(d, generator=g) * 0.1).to(DEV)
    layers = 3  # the batched K|V buffer of several decoder layers: [B, S, layers * 2d]
    kv_all = torch.randn(B, S, layers * 2 * d, generator=g).to(torch.bfloat16).to(DEV)
    kv5 = kv_all[:, :, 2 * d:4 * d].view(B, S, 2, H, hd)
    lens = torch.randint(1, S + 1, (B,), generator=g) if pad else None
    if pad:
        lens[0] = 0
    kv = lens.to(torch.int32).to(DEV) if pad else None
    scale = 1.0 / math.sqrt(hd)
    r = kk.qkv_attn_fwd(x, w, b, B, H, kv, scale, False, k=kv5[:, :, 0], v=kv5[:, :, 1])
    assert r is not None
    q, o, lse = r
    q0 = kk.linear_fwd(x, w, b)
    o0, lse0 = kk.attn_fwd(q0.view(B, T, H, hd), kv5[:, :, 0], kv5[:, :, 1], kv, scale, False)
    torch.cuda.synchronize()
    assert torch.equal(q, q0)
    if T > 64 or S <= 64:
        assert torch.equal(o, o0), f"O differs: {(o.float() - o0.float()).abs().max().item()}"
        assert torch.equal(lse, lse0)
    else:
        # (attn_fwd takes <= 64 queries in 64-key tiles with the online-softmax
        # rescale, the fused kernel all keys in one tile: rounding differs)
        assert (o.float() - o0.float()).abs().max().item() <= 1e-2 * o0.float().abs().max().item()
        assert (lse - lse0).abs().max().item() <= 1e-4 * lse0[lse0.isfinite()].abs().max().item()
