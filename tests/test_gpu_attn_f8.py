"""fp8 attention backward (attention.hip attn_bwd_f8_kernel): e4m3 Q/K/V/P,
e5m2 dO/dS on the fp8 MFMAs, checked against fp32 autograd of attention on
the dequantised operands (the e4m3 Q/K/V the forward ran on and the e5m2 dO
the kernel reads), plus its e5m2 outputs, amax records and bias-gradient
column sums against the bf16 outputs of the same call."""
import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import fp8 as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ref(q, k, v, kv_len, causal, scale):
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    Lq, Lk = q.shape[1], k.shape[1]
    mask = torch.zeros(q.shape[0], 1, Lq, Lk, dtype=torch.bool, device=q.device)
    if kv_len is not None:
        mask |= (torch.arange(Lk, device=q.device)[None, :] >= kv_len[:, None].long())[:, None, None, :]
    if causal:
        mask |= torch.ones(Lq, Lk, dtype=torch.bool, device=q.device).triu(1)[None, None]
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("bhqk,bkhd->bqhd", p, v)


def _setup(B, H, Lq, Lk, causal, seed, kv):
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    torch.manual_seed(seed)
    hd = 64
    meta, gmeta = F.Fp8Meta(DEV), F.Fp8Meta(DEV, fmt=1)
    slots = [meta.slot(n) for n in "qkv"]
    raw = [torch.randn(B, L, H, hd, device=DEV).bfloat16() * 2 for L in (Lq, Lk, Lk)]
    for t, i in zip(raw, slots):  # delayed scaling: amax -> power-of-two scale
        F.quantize(t, meta, i)
    meta.update()
    x8 = [F.quantize(t, meta, i, record=False).view(t.shape) for t, i in zip(raw, slots)]
    deq = [t8.float() / meta.scale[i].item() for t8, i in zip(x8, slots)]
    kv_len = torch.tensor([Lk, max(1, Lk - 37)][:B], dtype=torch.int32, device=DEV) if kv else None
    scale = hd ** -0.5
    o, lse = kk.attn_fwd_fp8(x8[0], x8[1], x8[2], meta.s(slots[0]), meta.s(slots[1]),
                             meta.s(slots[2]), kv_len, scale, causal)
    ido, ids, ig = gmeta.slot("do"), gmeta.slot("ds"), gmeta.slot("g")
    gmeta.scale.fill_(65536.0)
    do = (torch.randn(B, Lq, H, hd, device=DEV) * 0.01).bfloat16()
    F.quantize(do, gmeta, ido)
    gmeta.update()
    do8 = F.quantize(do, gmeta, ido, record=False).view(do.shape)
    do_deq = do8.float() / gmeta.scale[ido].item()
    return kk, meta, gmeta, slots, x8, deq, kv_len, scale, o, lse, (ido, ids, ig), do8, do_deq


def _run(kk, meta, gmeta, slots, x8, o, lse, kv_len, scale, causal, gs, do8, outs, part=None,
         cs=(0, 0, 0, 0)):
    ido, ids, ig = gs
    return kk.attn_bwd_f8(x8[0], x8[1], x8[2], meta.s(slots[0]), meta.s(slots[1]), meta.s(slots[2]),
                          o, do8, gmeta.s(ido), lse, kv_len, scale, causal, gmeta.s(ids),
                          gmeta.a(ids), *outs, sg8=gmeta.s(ig), amaxg8=gmeta.a(ig), cs_part=part,
                          cs_ld=cs[0], cs_q=cs[1], cs_k=cs[2], cs_v=cs[3])


@pytest.mark.parametrize("causal,Lq,Lk,kv", [(False, 384, 384, True), (True, 512, 512, False),
                                             (False, 260, 390, True), (True, 200, 200, True),
                                             (False, 512, 512, False)])
def test_attn_bwd_f8_matches_fp32_autograd(causal, Lq, Lk, kv):
    B, H, hd = 2, 3, 64
    (kk, meta, gmeta, slots, x8, deq, kv_len, scale, o, lse, gs, do8,
     do_deq) = _setup(B, H, Lq, Lk, causal, 7, kv)
    dq = torch.empty(B, Lq, H, hd, dtype=torch.bfloat16, device=DEV)
    dk = torch.empty(B, Lk, H, hd, dtype=torch.bfloat16, device=DEV)
    dv = torch.empty_like(dk)
    outs = (dq, dk, dv, None, None, None)
    # first call records the dS amax under the initial scale; the delayed
    # scale then sets the second call's e5m2 dS range
    _run(kk, meta, gmeta, slots, x8, o, lse, kv_len, scale, causal, gs, do8, outs)
    gmeta.update()
    assert 0 < gmeta.scale[gs[1]].item() < float("inf")
    _run(kk, meta, gmeta, slots, x8, o, lse, kv_len, scale, causal, gs, do8, outs)
    torch.cuda.synchronize()
    qr, kr, vr = (d.clone().requires_grad_(True) for d in deq)
    ref = _ref(qr, kr, vr, kv_len, causal, scale)
    ref.backward(do_deq)
    for name, got, want in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        g, w_ = got.float(), want
        assert torch.isfinite(g).all(), name
        rel = (g - w_).norm().item() / (w_.norm().item() + 1e-20)
        mx = (g - w_).abs().max().item() / (w_.abs().max().item() + 1e-20)
        # e4m3 P and e5m2 dS (2 mantissa bits) in the products: a few % in
        # norm; an indexing or layout error shows as O(1)
        assert rel < 0.08 and mx < 0.2, (name, rel, mx)


def test_attn_bwd_f8_e5m2_outputs_and_column_sums():
    """The e5m2 dq8/dk8/dv8 are e5m2(bf16(grad) * sg8) of the same call's bf16
    outputs, the gradient amax is recorded, and the per-batch column sums are
    those of the bf16-rounded gradients."""
    B, H, hd, L = 2, 3, 64, 320
    (kk, meta, gmeta, slots, x8, deq, kv_len, scale, o, lse, gs, do8,
     _) = _setup(B, H, L, L, True, 3, True)
    ig = gs[2]
    gmeta.scale[ig] = 2.0 ** 10
    dqkv = torch.empty(B, L, 3, H, hd, dtype=torch.bfloat16, device=DEV)
    d8 = torch.empty(B, L, 3, H, hd, dtype=torch.float8_e5m2, device=DEV)
    ld = 3 * H * hd
    part = torch.full((B, ld), float("nan"), device=DEV)
    outs = (dqkv[:, :, 0], dqkv[:, :, 1], dqkv[:, :, 2], d8[:, :, 0], d8[:, :, 1], d8[:, :, 2])
    n = _run(kk, meta, gmeta, slots, x8, o, lse, kv_len, scale, True, gs, do8, outs, part,
             (ld, 0, H * hd, 2 * H * hd))
    assert n == B
    torch.cuda.synchronize()
    want8 = (dqkv.float() * gmeta.scale[ig]).to(torch.float8_e5m2)
    assert torch.equal(d8.view(torch.uint8), want8.view(torch.uint8))
    sums = dqkv.float().sum(1).reshape(B, ld)
    assert torch.allclose(part, sums, rtol=1e-4, atol=1e-4 * sums.abs().max().item())
    amax = gmeta.amax_values()[ig].item()
    assert amax == pytest.approx(dqkv.float().abs().max().item(), rel=1e-6)
    assert gmeta.amax_values()[gs[1]].item() > 0  # dS amax recorded


def test_attn_bwd_f8_only_e5m2_dq_bf16_dkdv():
    """The cross-attention form: e5m2 dQ (bias sums at column 0) with bf16
    dK / dV only; equals the all-outputs call."""
    B, H, hd, Lq, Lk = 2, 3, 64, 300, 400
    (kk, meta, gmeta, slots, x8, deq, kv_len, scale, o, lse, gs, do8,
     _) = _setup(B, H, Lq, Lk, False, 5, True)
    dq = torch.empty(B, Lq, H, hd, dtype=torch.bfloat16, device=DEV)
    dk = torch.empty(B, Lk, H, hd, dtype=torch.bfloat16, device=DEV)
    dv = torch.empty_like(dk)
    dq8 = torch.empty(B, Lq, H, hd, dtype=torch.float8_e5m2, device=DEV)
    _run(kk, meta, gmeta, slots, x8, o, lse, kv_len, scale, False, gs, do8,
         (dq, dk, dv, dq8, None, None))
    dk2, dv2 = torch.empty_like(dk), torch.empty_like(dv)
    dq82 = torch.empty_like(dq8)
    part = torch.zeros(B, H * hd, device=DEV)
    _run(kk, meta, gmeta, slots, x8, o, lse, kv_len, scale, False, gs, do8,
         (None, dk2, dv2, dq82, None, None), part, (H * hd, 0, 0, 0))
    torch.cuda.synchronize()
    assert torch.equal(dk, dk2) and torch.equal(dv, dv2)
    assert torch.equal(dq8.view(torch.uint8), dq82.view(torch.uint8))
    assert torch.allclose(part, dq.float().sum(1).reshape(B, -1), rtol=1e-4, atol=1e-5)


def test_attn_bwd_f8_cross_kv_own_slot_and_column_sums():
    """The form the fp8 step runs for cross-attention by default (KVGrad.f8b):
    e5m2 dQ in the Q-projection gradient slot (sg8 / amaxg8, column sums at
    cs_q of cs_part) and e5m2 dK / dV written straight into a layer's slice of
    the batched cross K|V gradient [B, Lk, layers * 2d] in that projection's
    own slot (sgkv8 / amaxgkv8, a different scale), their column sums at the
    layer's offsets cs_k / cs_v of the wider cs_part2. Every output is checked
    against the bf16 gradients of the same call."""
    B, H, hd, Lq, Lk = 2, 3, 64, 300, 400
    d = H * hd
    layers, layer = 3, 1
    NKV = layers * 2 * d
    (kk, meta, gmeta, slots, x8, deq, kv_len, scale, o, lse, gs, do8,
     _) = _setup(B, H, Lq, Lk, False, 9, True)
    ido, ids, ig = gs
    ikv = gmeta.slot("gkv")
    gmeta.scale[ig] = 2.0 ** 10
    gmeta.scale[ikv] = 2.0 ** 13  # != sg8: a wrong slot shows in every byte
    dq = torch.empty(B, Lq, H, hd, dtype=torch.bfloat16, device=DEV)
    # (the bf16 and e5m2 outputs share strides: both batched [B, Lk, NKV])
    bufb = torch.zeros(B, Lk, NKV, dtype=torch.bfloat16, device=DEV)
    gb5 = bufb[:, :, layer * 2 * d:(layer + 1) * 2 * d].view(B, Lk, 2, H, hd)
    dk, dv = gb5[:, :, 0], gb5[:, :, 1]
    dq8 = torch.empty(B, Lq, H, hd, dtype=torch.float8_e5m2, device=DEV)
    buf8 = torch.zeros(B, Lk, NKV, dtype=torch.float8_e5m2, device=DEV)
    g85 = buf8[:, :, layer * 2 * d:(layer + 1) * 2 * d].view(B, Lk, 2, H, hd)
    part = torch.full((B, d), float("nan"), device=DEV)
    part2 = torch.full((B, NKV), float("nan"), device=DEV)
    n = kk.attn_bwd_f8(x8[0], x8[1], x8[2], meta.s(slots[0]), meta.s(slots[1]), meta.s(slots[2]),
                       o, do8, gmeta.s(ido), lse, kv_len, scale, False, gmeta.s(ids), gmeta.a(ids),
                       dq=dq, dk=dk, dv=dv, dq8=dq8, dk8=g85[:, :, 0], dv8=g85[:, :, 1],
                       sg8=gmeta.s(ig), amaxg8=gmeta.a(ig), cs_part=part, cs_ld=d, cs_q=0,
                       sgkv8=gmeta.s(ikv), amaxgkv8=gmeta.a(ikv), cs_part2=part2, cs_ld2=NKV,
                       cs_k=layer * 2 * d, cs_v=layer * 2 * d + d)
    assert n == B
    torch.cuda.synchronize()

    def e5(x, s):
        return (x.float() * s).clamp(-57344, 57344).to(torch.float8_e5m2).view(torch.uint8)

    assert torch.equal(dq8.view(torch.uint8), e5(dq, 2.0 ** 10))
    assert torch.equal(g85[:, :, 0].contiguous().view(torch.uint8), e5(dk, 2.0 ** 13))
    assert torch.equal(g85[:, :, 1].contiguous().view(torch.uint8), e5(dv, 2.0 ** 13))
    # the other layers' slices of the batched buffer are untouched
    other = torch.cat([buf8[:, :, :layer * 2 * d], buf8[:, :, (layer + 1) * 2 * d:]], -1)
    assert int(other.view(torch.uint8).count_nonzero()) == 0
    # separate amax slots
    am = gmeta.amax_values()
    assert am[ig].item() == pytest.approx(dq.float().abs().max().item(), rel=1e-6)
    assert am[ikv].item() == pytest.approx(max(dk.float().abs().max().item(),
                                               dv.float().abs().max().item()), rel=1e-6)
    # column sums: dQ's in cs_part, dK / dV's at the layer's offsets of cs_part2
    assert torch.allclose(part, dq.float().sum(1).reshape(B, d), rtol=1e-4, atol=1e-5)
    for off, g in ((layer * 2 * d, dk), (layer * 2 * d + d, dv)):
        want = g.float().sum(1).reshape(B, d)
        assert torch.allclose(part2[:, off:off + d], want, rtol=1e-4, atol=1e-4 * want.abs().max().item())
