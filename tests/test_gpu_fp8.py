"""FP8 (OCP e4m3 / e5m2) path: quantisation vs torch's float8 types, the
block-scaled MFMA GEMM (forward, and the e5m2-gradient backward GEMMs with the
ReLU-backward mask and beta accumulation) vs an fp32 reference of the
dequantised operands, the fused fp8 epilogue output, delayed scaling, and an
fp8 training run (forward + FFN backward in fp8) vs bf16."""
import math

import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import fp8 as F
from tensorflow_distributed_on_gke_amd.ops._ext import C

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_quantize_matches_torch_e4m3():
    meta = F.Fp8Meta(DEV)
    i = meta.slot("x")
    meta.scale[i] = 37.0
    x = (torch.randn(1000, 96, device=DEV) * 3).bfloat16()
    x[0, 0] = 100.0  # saturates at 448 after scaling
    x8 = F.quantize(x, meta, i)
    ref = (x.float() * 37.0).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (x8.view(torch.uint8) == ref.view(torch.uint8)).float().mean().item() > 0.999
    assert abs(meta.amax_values()[i].item() - x.float().abs().max().item()) < 1e-6
    meta.update()
    # power-of-two delayed scale: the largest 2^k <= 448 / amax
    r = 448.0 / x.float().abs().max().item()
    assert meta.scale[i].item() == 2.0 ** math.floor(math.log2(r))
    assert meta.amax_values()[i].item() == 0.0


@pytest.mark.parametrize("M,N,K", [(512, 384, 256), (333, 1000, 512), (8192, 2048, 512), (64, 64, 128),
                                   (700, 600, 1024)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_fp8(M, N, K, epi):
    torch.manual_seed(0)
    meta = F.Fp8Meta(DEV)
    ia, ib, io = meta.slot("a"), meta.slot("b"), meta.slot("o")
    meta.scale[ia], meta.scale[ib], meta.scale[io] = 60.0, 900.0, 4.0
    a = torch.randn(M, K, device=DEV).bfloat16()
    b = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(N, device=DEV) if epi else None
    a8, b8 = F.quantize(a, meta, ia), F.quantize(b, meta, ib)
    ref = (a8.float() / 60.0) @ (b8.float() / 900.0).t()
    if epi:
        ref = ref + bias
    if epi == 2:
        ref = ref.relu()
    for cfg in F._CANDS:
        y, y8 = F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=epi == 2, out8_slot=io, cfg=cfg)
        err = (y.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
        assert err < 1e-2, (cfg, err)
        want8 = (y.float() * 4.0).clamp(-448, 448).to(torch.float8_e4m3fn)
        assert (y8.view(torch.uint8) == want8.view(torch.uint8)).float().mean().item() > 0.999
    assert abs(meta.amax_values()[io].item() - y.float().abs().max().item()) <= 1e-3 * y.float().abs().max().item()


def test_quantize_matches_torch_e5m2():
    meta = F.Fp8Meta(DEV, fmt=1)
    i = meta.slot("g")
    meta.scale[i] = 4096.0
    x = (torch.randn(1000, 96, device=DEV) * 1e-3).bfloat16()
    x[0, 0] = 30.0  # saturates at 57344 after scaling
    x8 = F.quantize(x, meta, i)
    assert x8.dtype == torch.float8_e5m2
    ref = (x.float() * 4096.0).clamp(-57344, 57344).to(torch.float8_e5m2)
    assert (x8.view(torch.uint8) == ref.view(torch.uint8)).float().mean().item() > 0.999
    meta.update()
    assert meta.scale[i].item() == 2.0 ** math.floor(math.log2(57344.0 / 30.0))


@pytest.mark.parametrize("M,N,K", [(512, 384, 256), (333, 1000, 512), (64, 64, 128), (600, 520, 1024)])
@pytest.mark.parametrize("relu,beta", [(True, 0.0), (False, 1.0)])
@pytest.mark.parametrize("cfg", [0, 9, 10, "plain", "plain10"])
def test_gemm_bf8_dgrad(M, N, K, relu, beta, cfg):
    """out (=|+= beta) dequant(g8 e5m2 @ w8t e4m3^T), ReLU-backward mask, and
    the e5m2 copy of the output, against an fp32 reference. "plain": the
    weight given untransposed ([K][N], read N-contiguous by the kernel);
    10: the half-stage ring kernel."""
    if str(cfg).startswith("plain") and N % 16:
        pytest.skip("the N-contiguous weight path needs N % 16 == 0")
    torch.manual_seed(1)
    wm, gm = F.Fp8Meta(DEV), F.Fp8Meta(DEV, fmt=1)
    iw, ig, io = wm.slot("w"), gm.slot("g"), gm.slot("o")
    wm.scale[iw], gm.scale[ig], gm.scale[io] = 900.0, 2.0 ** 20, 2.0 ** 10
    g = (torch.randn(M, K, device=DEV) * 1e-3).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    aux = torch.randn(M, N, device=DEV).bfloat16() if relu else None
    out = torch.randn(M, N, device=DEV).bfloat16()
    g8, w8 = F.quantize(g, gm, ig), F.quantize(w, wm, iw)
    ref = (g8.float() / 2.0 ** 20) @ (w8.float() / 900.0).t()
    if relu:
        ref = ref * (aux.float() > 0)
    ref = ref + beta * out.float()
    if str(cfg).startswith("plain"):
        o8 = F.gemm_bf8_dgrad(g8, gm, ig, w8.t().contiguous(), wm, iw, out, relu_aux=aux, beta=beta,
                              out8_slot=io if relu else None, w_plain=True,
                              cfg=10 if cfg == "plain10" else 0)
    else:
        o8 = F.gemm_bf8_dgrad(g8, gm, ig, w8, wm, iw, out, relu_aux=aux, beta=beta,
                              out8_slot=io if relu else None, cfg=cfg)
    err = (out.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)
    assert err < 1e-2, err
    if relu:
        want = (out.float() * 2.0 ** 10).clamp(-57344, 57344).to(torch.float8_e5m2)
        assert (o8.view(torch.uint8) == want.view(torch.uint8)).float().mean().item() > 0.999
        assert abs(gm.amax_values()[io].item() - out.float().abs().max().item()) <= 1e-3 * out.float().abs().max().item()


def test_fp8_training_tracks_bf16():
    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    cfg = model_config("tiny", src_vocab=64, tgt_vocab=64, dropout=0.0)
    data = SyntheticPairs(batch=32, src_len=16, tgt_len=17, src_vocab=64, tgt_vocab=64, copy_task=True, seed=0)
    finals = {}
    for mode in ("bf16", "fp8"):
        m = Transformer(cfg).build("cuda", seed=1)
        opt = Adam(m.store, cfg.d_model, lr=1e-3)
        st = F.Fp8State(m) if mode == "fp8" else None
        step = TrainStep(m, opt, None, workers=1.0, seed=3, fp8_state=st)
        losses = []
        for i in range(150):
            src, tgt = data.batch(i)
            losses.append(step(src.cuda(), tgt.cuda())[0].item())
        finals[mode] = (losses[0], sum(losses[-10:]) / 10)
    (b0, b1), (f0, f1) = finals["bf16"], finals["fp8"]
    assert b1 < 0.75 * b0 and f1 < 0.75 * f0, finals
    assert abs(f1 - b1) < 0.1 * b1 + 0.05, finals


@pytest.mark.parametrize("D", [128, 512, 1024])
def test_layernorm_fused_fp8_copy(D):
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    meta = F.Fp8Meta(DEV)
    i = meta.slot("y")
    meta.scale[i] = 50.0
    x = torch.randn(777, D, device=DEV).bfloat16()
    s = torch.randn(777, D, device=DEV).bfloat16()
    g, b = torch.rand(D, device=DEV) + 0.5, torch.randn(D, device=DEV)
    y8 = torch.empty(777, D, dtype=F.FP8, device=DEV)
    y, *_ = kk.ln_fwd(x, s, g, b, 0.0, 0, None, 0, y8=y8, s8=meta.s(i), amax8=meta.a(i))
    want = (y.float() * 50.0).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert (y8.view(torch.uint8) == want.view(torch.uint8)).float().mean().item() > 0.999
    assert abs(meta.amax_values()[i].item() - y.float().abs().max().item()) < 1e-6 * D


def _attn_ref(q, k, v, kv_len, causal, scale):
    """fp32 attention with the reference's -1e9 mask add (kv_len = 0 rows:
    uniform over all keys); O and the log2-domain log-sum-exp."""
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    B, H, Lq, Lk = s.shape
    keys = torch.arange(Lk, device=q.device)
    mask = (keys.view(1, 1, 1, Lk) >= kv_len.view(B, 1, 1, 1)).float().expand(B, 1, Lq, Lk)
    if causal:
        la = (keys.view(1, Lk) > torch.arange(Lq, device=q.device).view(Lq, 1)).float()
        mask = torch.maximum(mask, la.view(1, 1, Lq, Lk))
    s = s + mask * -1e9
    p = torch.softmax(s, -1)
    lse2 = torch.logsumexp(s, -1) / 0.6931471805599453
    return torch.einsum("bhqk,bkhd->bqhd", p, v), lse2


@pytest.mark.parametrize("causal,Lq,Lk", [(False, 512, 512), (True, 512, 512), (False, 260, 390),
                                          (False, 200, 70), (True, 300, 300), (True, 700, 700)])
def test_attention_fwd_fp8(causal, Lq, Lk):
    """e4m3 attention forward (attention.hip attn_fwd_fp8_kernel) against fp32 attention of the dequantised e4m3 inputs: the error
    left is the e4m3 rounding of P. Ragged key lengths and a kv_len = 0 row
    (non-causal)."""
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    torch.manual_seed(5)
    B, H, hd = 3, 2, 64
    q, k, v = (torch.randn(B, L, H, hd, device=DEV).bfloat16() for L in (Lq, Lk, Lk))
    kv_len = torch.tensor([Lk, 0 if not causal else Lk // 2, max(1, Lk - 5)], dtype=torch.int32, device=DEV)
    sc = [torch.tensor([448.0 / t.float().abs().max().item()], device=DEV) for t in (q, k, v)]
    q8, k8, v8 = ((t.float() * s).clamp(-448, 448).to(torch.float8_e4m3fn) for t, s in zip((q, k, v), sc))
    scale = hd ** -0.5
    out, lse = kk.attn_fwd_fp8(q8, k8, v8, sc[0], sc[1], sc[2], kv_len, scale, causal)
    qd, kd, vd = (t8.float() / s for t8, s in zip((q8, k8, v8), sc))
    ref, lref = _attn_ref(qd, kd, vd, kv_len, causal, scale)
    err = (out.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 4e-2, err
    live = kv_len > 0  # (kv_len = 0 rows: the kernel's LSE is of its own zero-scale logits)
    lerr = (lse[live] - lref[live]).abs().max().item()
    assert lerr < 2e-2, lerr
    # and close to the bf16 kernel on the unquantised inputs
    ob, _ = kk.attn_fwd(q, k, v, kv_len, scale, causal)
    assert (out.float() - ob.float()).abs().max().item() < 0.15 * ob.float().abs().max().item()
    # the epilogue's e4m3 copy of O equals quantising the bf16 O; amax recorded
    meta = F.Fp8Meta(DEV)
    io = meta.slot("o")
    meta.scale[io] = 64.0
    o8 = torch.empty(out.shape, dtype=torch.float8_e4m3fn, device=DEV)
    out2, _ = kk.attn_fwd_fp8(q8, k8, v8, sc[0], sc[1], sc[2], kv_len, scale, causal, o8, meta.s(io),
                              meta.a(io))
    assert torch.equal(out2, out)
    want = (out.float() * 64.0).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(o8.view(torch.uint8), want.view(torch.uint8))
    assert meta.amax_values()[io].item() == out.float().abs().max().item()


def test_fp8_attention_training_tracks_bf16(monkeypatch):
    """fp8 mode with e4m3 attention (hd 64, sequences > 128: the input
    projections emit e4m3 Q|K|V, attn_fwd_fp8 consumes them, the fp8
    attention backward attn_bwd_f8 runs on them and an e5m2 dO) trains like
    bf16 on the copy task."""
    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    calls = {"n": 0, "bwd": 0}
    real, real_bwd = kk.attn_fwd_fp8, kk.attn_bwd_f8

    def counting(*a, **k):
        calls["n"] += 1
        return real(*a, **k)

    def counting_bwd(*a, **k):
        calls["bwd"] += 1
        return real_bwd(*a, **k)

    monkeypatch.setattr(kk, "attn_fwd_fp8", counting)
    monkeypatch.setattr(kk, "attn_bwd_f8", counting_bwd)
    cfg = model_config("tiny", heads=2, src_vocab=64, tgt_vocab=64, dropout=0.0)
    data = SyntheticPairs(batch=8, src_len=160, tgt_len=161, src_vocab=64, tgt_vocab=64, copy_task=True, seed=0)
    finals = {}
    for mode in ("bf16", "fp8"):
        m = Transformer(cfg).build("cuda", seed=1)
        opt = Adam(m.store, cfg.d_model, lr=1e-3)
        st = F.Fp8State(m) if mode == "fp8" else None
        step = TrainStep(m, opt, None, workers=1.0, seed=3, fp8_state=st)
        losses = []
        for i in range(120):
            src, tgt = data.batch(i)
            losses.append(step(src.cuda(), tgt.cuda())[0].item())
        finals[mode] = (losses[0], sum(losses[-10:]) / 10)
    assert calls["n"] > 0, "e4m3 attention did not run"
    assert calls["bwd"] > 0 or not F.ATTN_BWD_F8, "the fp8 attention backward did not run"
    (b0, b1), (f0, f1) = finals["bf16"], finals["fp8"]
    assert b1 < 0.9 * b0 and f1 < 0.9 * f0, finals  # (long copy task: slower start)
    assert abs(f1 - b1) < 0.1 * b1 + 0.05, finals


def test_quant_multi_matches_single():
    """The weight refresh's one-launch quantisation of many tensors is bitwise
    the per-tensor quantisation, with each tensor's amax in its own slot."""
    torch.manual_seed(3)
    meta = F.Fp8Meta(DEV)
    shapes = [(1024, 1024), (7, 13), (4096, 1024), (3, 8), (1000, 512)]
    xs = [(torch.randn(*s, device=DEV) * (i + 1)).bfloat16() for i, s in enumerate(shapes)]
    slots = [meta.slot(f"w{i}") for i in range(len(xs))]
    for i, s in enumerate(slots):
        meta.scale[s] = 448.0 / (i + 1) / 5.0
    want = [F.quantize(x, meta, s, record=False) for x, s in zip(xs, slots)]
    got = [torch.empty_like(w) for w in want]
    from tensorflow_distributed_on_gke_amd.ops._ext import C
    C().fp8_quant_multi(xs, got, slots, meta.scale, meta.amax)
    for g, w in zip(got, want):
        assert torch.equal(g.view(torch.uint8), w.view(torch.uint8))
    am = meta.amax_values()
    for x, s in zip(xs, slots):
        assert am[s].item() == x.float().abs().max().item()


@pytest.mark.parametrize("relu", [False, True])
def test_gemm_fp8_c_deq(relu):
    """c_deq: the bf16 output is exactly dequant(y8) (power-of-two scale), and
    y8 is unchanged by the flag."""
    torch.manual_seed(2)
    meta = F.Fp8Meta(DEV)
    ia, ib, io = meta.slot("a"), meta.slot("b"), meta.slot("o")
    meta.scale[ia], meta.scale[ib], meta.scale[io] = 64.0, 1024.0, 8.0
    a = torch.randn(1000, 256, device=DEV).bfloat16()
    b = (torch.randn(384, 256, device=DEV) * 0.05).bfloat16()
    bias = torch.randn(384, device=DEV)
    a8, b8 = F.quantize(a, meta, ia), F.quantize(b, meta, ib)
    y0, y80 = F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=relu, out8_slot=io, cfg=0)
    y, y8 = F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=relu, out8_slot=io, cfg=0, c_deq=True)
    assert torch.equal(y8.view(torch.uint8), y80.view(torch.uint8))
    assert torch.equal(y.float(), y8.float() / 8.0)
    # and within e4m3 rounding of the plain output
    assert (y.float() - y0.float()).abs().max().item() <= 0.07 * y0.float().abs().max().item()


@pytest.mark.parametrize("causal,Lq,Lk", [(False, 384, 384), (True, 512, 512), (False, 260, 390)])
def test_fp8_attention_gradients_consistent(causal, Lq, Lk):
    """fp8 mode's attention: forward on e4m3 Q/K/V (attn_fwd_fp8), backward
    (attn_bwd) on the bf16 copies the c_deq projection epilogue writes, i.e.
    the dequantised e4m3 values. The gradients must be those of fp32
    attention on the dequantised inputs -- the backward's recomputed P must
    match the P of the forward that produced O and the LSE."""
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    torch.manual_seed(7)
    B, H, hd = 2, 3, 64
    meta = F.Fp8Meta(DEV)
    slots = [meta.slot(n) for n in "qkv"]
    raw = [torch.randn(B, L, H, hd, device=DEV).bfloat16() * 2 for L in (Lq, Lk, Lk)]
    for t, i in zip(raw, slots):  # delayed scaling: amax -> power-of-two scale
        F.quantize(t, meta, i)
    meta.update()
    x8 = [F.quantize(t, meta, i, record=False).view(t.shape) for t, i in zip(raw, slots)]
    sc = [meta.scale[i].item() for i in slots]
    deq = [(t8.float() / s) for t8, s in zip(x8, sc)]
    q, k, v = (d.bfloat16() for d in deq)
    for d, bq in zip(deq, (q, k, v)):
        assert torch.equal(d, bq.float())  # exact: power-of-two scales
    kv_len = torch.tensor([Lk, max(1, Lk - 37)], dtype=torch.int32, device=DEV)
    scale = hd ** -0.5
    o, lse = kk.attn_fwd_fp8(x8[0], x8[1], x8[2], meta.s(slots[0]), meta.s(slots[1]),
                             meta.s(slots[2]), kv_len, scale, causal)
    do = torch.randn(B, Lq, H, hd, device=DEV).bfloat16()
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    kk.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, kv_len, scale, causal)
    qr, kr, vr = (d.clone().requires_grad_(True) for d in deq)
    ref, _ = _attn_ref(qr, kr, vr, kv_len, causal, scale)
    ref.backward(do.float())
    for name, got, want in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        err = (got.float() - want).abs().max().item() / (want.abs().max().item() + 1e-12)
        # bf16 kernels on exact operands: the forward's e4m3 P and bf16 O are
        # the only roundings left (a P inconsistent with the forward's LSE
        # shows as errors of order 1)
        assert err < 5e-2, (name, err)


@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_wgrad_fp8_ragged(beta):
    """fp8 weight gradients (transposing-read TN kernel): e5m2 dY^T x e4m3 X
    over tokens, several shape classes in one launch (incl. a strided view and
    a non-multiple-of-256 size), against fp32 of the dequantised operands."""
    torch.manual_seed(11)
    T = 1024
    specs = [(1024, 256), (1024, 256), (256, 1024), (512, 512), (272, 400)]
    gm, am = F.Fp8Meta(DEV, fmt=1), F.Fp8Meta(DEV)
    dys, xs, dws, sas, sbs, refs = [], [], [], [], [], []
    for i, (M, N) in enumerate(specs):
        ga, ab = gm.slot(f"g{i}"), am.slot(f"x{i}")
        gm.scale[ga], am.scale[ab] = 2.0 ** (12 + i % 3), 2.0 ** (4 - i % 2)
        ld = M + 64 if i == 3 else M
        dy = (torch.randn(T, ld, device=DEV) * 1e-3).bfloat16()
        x = torch.randn(T, N, device=DEV).bfloat16()
        dy8 = F.quantize(dy, gm, ga).view(T, ld)[:, :M]
        x8 = F.quantize(x, am, ab).view(T, N)
        dw = torch.randn(M, N, device=DEV)
        refs.append((dy8.float() / gm.scale[ga]).t() @ (x8.float() / am.scale[ab]) + beta * dw)
        dys.append(dy8), xs.append(x8), dws.append(dw), sas.append(gm.s(ga)), sbs.append(am.s(ab))
    F.wgrad_fp8(dys, sas, xs, sbs, dws, beta)
    for i, (dw, ref) in enumerate(zip(dws, refs)):
        err = (dw - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)
        assert err < 1e-4, (i, specs[i], err)


def test_fp8_ffn_wgrad_matches_bf16_path(monkeypatch):
    """The FFN weight gradients of an fp8 step: fp8 path vs the bf16 ragged
    path on the same (e4m3-rounded) forward -- within fp8 gradient noise."""
    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.models.layers import RunCtx, WgradQueue

    cfg = model_config("tiny", src_vocab=64, tgt_vocab=64, dropout=0.0)
    data = SyntheticPairs(batch=16, src_len=16, tgt_len=17, src_vocab=64, tgt_vocab=64, copy_task=True, seed=0)
    src, tgt = (t.cuda() for t in data.batch(0))
    grads = {}
    for mode in (False, True):
        monkeypatch.setattr(F, "WGRAD_FP8", mode)
        m = Transformer(cfg).build("cuda", seed=1)
        st = F.Fp8State(m)
        rt = RunCtx(training=True, dropout=0.0, seed=3, store=m.store, fp8=st,
                    ctr=torch.zeros(1, dtype=torch.int64, device="cuda"))
        rt.wgrad = WgradQueue()
        rt.wgrad.layers_per_step = 2 * cfg.layers
        m.loss_and_backward(src, tgt, rt, 1.0)
        torch.cuda.synchronize()
        grads[mode] = {n: p.grad.clone() for n, p in ((l.ff1.w.name, l.ff1.w) for l in m.enc_layers)}
        grads[mode].update({l.ff2.w.name: l.ff2.w.grad.clone() for l in m.enc_layers})
    for n, g16 in grads[False].items():
        g8 = grads[True][n]
        rel = ((g8 - g16).norm() / g16.norm()).item()
        assert rel < 0.1, (n, rel)


@pytest.mark.parametrize("M,N,K", [(512, 384, 256), (333, 1000, 512), (1024, 4096, 1024)])
@pytest.mark.parametrize("with_c", [True, False])
@pytest.mark.parametrize("plain", [False, True])
@pytest.mark.parametrize("cfg", [0, 10])
def test_gemm_bf8_dgrad_mask8_colsum(M, N, K, with_c, plain, cfg):
    """The lean fp8 FFN backward's ReLU-backward dgrad: mask from the e4m3
    hidden (h8 != 0), optional bf16 output, e5m2 copy, and the bias gradient
    (column sums of the bf16-rounded output, accumulated with beta) from the
    epilogue partials."""
    if plain and N % 16:
        pytest.skip("the N-contiguous weight path needs N % 16 == 0")
    torch.manual_seed(4)
    wm, gm = F.Fp8Meta(DEV), F.Fp8Meta(DEV, fmt=1)
    iw, ig, io, ih = wm.slot("w"), gm.slot("g"), gm.slot("o"), wm.slot("h")
    wm.scale[iw], gm.scale[ig], gm.scale[io], wm.scale[ih] = 512.0, 2.0 ** 20, 2.0 ** 10, 8.0
    g = (torch.randn(M, K, device=DEV) * 1e-3).bfloat16()
    w = (torch.randn(N, K, device=DEV) * 0.05).bfloat16()
    h = torch.relu(torch.randn(M, N, device=DEV)).bfloat16()
    h8 = F.quantize(h, wm, ih).view(M, N)
    g8, w8 = F.quantize(g, gm, ig), F.quantize(w, wm, iw)
    ref = ((g8.float() / 2.0 ** 20) @ (w8.float() / 512.0).t()) * (h8.float() != 0)
    out = torch.empty(M, N, device=DEV).bfloat16() if with_c else None
    bsum = torch.randn(N, device=DEV)
    bref = bsum + ref.bfloat16().float().sum(0)
    o8 = F.gemm_bf8_dgrad(g8, gm, ig, w8.t().contiguous() if plain else w8, wm, iw, out,
                          relu_aux8=h8, out8_slot=io, colsum_out=bsum, colsum_beta=1.0, w_plain=plain,
                          cfg=cfg)
    # (the kernel quantises the bf16-rounded value; compare values: masked
    # elements are +0 from the kernel, -0 in ref * 0)
    o8ref = (ref.bfloat16().float() * 2.0 ** 10).clamp(-57344, 57344).to(torch.float8_e5m2)
    assert (o8.float() == o8ref.float()).float().mean().item() > 0.995
    if with_c:
        err = (out.float() - ref).abs().max().item() / (ref.abs().max().item() + 1e-12)
        assert err < 1e-2, err
    berr = (bsum - bref).abs().max().item() / (bref.abs().max().item() + 1e-12)
    assert berr < 1e-3, berr


@pytest.mark.parametrize("D", [512, 1024])
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_ln_bwd_emits_e5m2_ds(D, p):
    """LayerNorm backward with the e5m2 copy of ds (the lean fp8 FFN
    backward): equal to quantising the bf16 ds, amax recorded, same dh and
    bias column sums as the bf16 path."""
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    torch.manual_seed(6)
    M = 1000
    x = torch.randn(M, D, device=DEV).bfloat16()
    s = torch.randn(M, D, device=DEV).bfloat16()
    g, b = torch.rand(D, device=DEV) + 0.5, torch.randn(D, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    y, h, mean, rstd = kk.ln_fwd(x, s, g, b, p, 7, ctr, 3)
    dy = torch.randn(M, D, device=DEV).bfloat16()
    gm = F.Fp8Meta(DEV, fmt=1)
    i = gm.slot("ds")
    gm.scale[i] = 2.0 ** 8
    outs = {}
    for mode in ("bf16", "e5m2"):
        dg, dbt, dbias = (torch.zeros(D, device=DEV) for _ in range(3))
        if mode == "bf16":
            dh, ds = kk.ln_bwd(dy, h, mean, rstd, g, dg, dbt, dbias, p, 7, ctr, 3)
        else:
            ds8 = torch.empty(M, D, dtype=F.BF8, device=DEV)
            dh, _ = kk.ln_bwd(dy, h, mean, rstd, g, dg, dbt, dbias, p, 7, ctr, 3, want_ds=False,
                              ds8=ds8, s8=gm.s(i), amax8=gm.a(i))
            ds = ds8
        outs[mode] = (dh.clone(), ds.clone(), dg, dbt, dbias)
    dh16, ds16, dg16, db16, bias16 = outs["bf16"]
    dh8, ds8, dg8, db8, bias8 = outs["e5m2"]
    assert torch.equal(dh16, dh8)
    assert torch.equal(dg16, dg8) and torch.equal(db16, db8)
    assert torch.allclose(bias16, bias8, rtol=1e-5, atol=1e-5)
    want = F.quantize(ds16, gm, i, record=False)
    assert (ds8.view(torch.uint8) == want.view(torch.uint8)).float().mean().item() > 0.999
    assert abs(gm.amax_values()[i].item() - ds16.float().abs().max().item()) <= 1e-6 * ds16.float().abs().max().item()


def test_fp8_attention_projection_grads_match_bf16_path(monkeypatch):
    """Attention projections in fp8 (e4m3 O-projection forward, e5m2 x e4m3
    dgrads and weight gradients of every projection) vs the same step with
    those projections in bf16: the projection weight / bias gradients agree
    within fp8 gradient noise, and the loss matches."""
    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.models.layers import RunCtx, WgradQueue

    cfg = model_config("tiny", src_vocab=64, tgt_vocab=64, dropout=0.0)
    data = SyntheticPairs(batch=16, src_len=16, tgt_len=17, src_vocab=64, tgt_vocab=64, copy_task=True, seed=0)
    src, tgt = (t.cuda() for t in data.batch(0))
    res = {}
    for mode in (False, True):
        monkeypatch.setattr(F, "ATTN_PROJ_FP8", mode)
        m = Transformer(cfg).build("cuda", seed=1)
        st = F.Fp8State(m)
        assert bool(st.attn_out) == mode
        rt = RunCtx(training=True, dropout=0.0, seed=3, store=m.store, fp8=st,
                    ctr=torch.zeros(1, dtype=torch.int64, device="cuda"))
        rt.wgrad = WgradQueue()
        rt.wgrad.layers_per_step = 2 * cfg.layers
        out = m.loss_and_backward(src, tgt, rt, 1.0)
        torch.cuda.synchronize()
        ps = []
        for l in m.enc_layers:
            ps += [l.qkv.w, l.qkv.b, l.o.w]
        for l in m.dec_layers:
            ps += [l.qkv1.w, l.q2.w, l.q2.b, l.o2.w]
        ps += [m.cross_kv.w, m.cross_kv.b]
        res[mode] = (float(out[0]), {p.name: p.grad.clone() for p in ps})
    (l16, g16), (l8, g8) = res[False], res[True]
    assert abs(l8 - l16) < 0.02 * abs(l16)
    for n, a in g16.items():
        rel = ((g8[n] - a).norm() / (a.norm() + 1e-12)).item()
        assert rel < 0.15, (n, rel)


def test_fp8_attention_backward_grads_match_bf16_backward(monkeypatch):
    """Sequences > 128 (the fp8 attention backward, and with it the e5m2
    cross K|V gradient written straight by the decoder layers' kernels) vs
    the same fp8 step with the bf16 attention backward: projection weight /
    bias gradients within fp8 gradient noise, same loss."""
    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.models.layers import RunCtx, WgradQueue

    cfg = model_config("tiny", heads=2, src_vocab=64, tgt_vocab=64, dropout=0.0)
    data = SyntheticPairs(batch=8, src_len=160, tgt_len=161, src_vocab=64, tgt_vocab=64, copy_task=True, seed=0)
    src, tgt = (t.cuda() for t in data.batch(0))
    res = {}
    for mode in (False, True):
        monkeypatch.setattr(F, "ATTN_BWD_F8", mode)
        m = Transformer(cfg).build("cuda", seed=1)
        st = F.Fp8State(m)
        rt = RunCtx(training=True, dropout=0.0, seed=3, store=m.store, fp8=st,
                    ctr=torch.zeros(1, dtype=torch.int64, device="cuda"))
        rt.wgrad = WgradQueue()
        rt.wgrad.layers_per_step = 2 * cfg.layers
        for _ in range(2):  # second step: delayed scales (dO, dS, gradients) calibrated
            m.store.zero_grad()
            out = m.loss_and_backward(src, tgt, rt, 1.0)
            st.after_step()
        torch.cuda.synchronize()
        ps = [m.cross_kv.w, m.cross_kv.b]
        for l in m.enc_layers:
            ps += [l.qkv.w, l.qkv.b]
        for l in m.dec_layers:
            ps += [l.qkv1.w, l.q2.w, l.q2.b]
        res[mode] = (float(out[0]), {p.name: p.grad.clone() for p in ps})
    (l16, g16), (l8, g8) = res[False], res[True]
    assert abs(l8 - l16) < 0.02 * abs(l16)
    for n, a in g16.items():
        assert torch.isfinite(g8[n]).all(), n
        rel = ((g8[n] - a).norm() / (a.norm() + 1e-12)).item()
        assert rel < 0.2, (n, rel)


@pytest.mark.parametrize("R,NC", [(1024, 3072), (300, 520), (64, 8)])
def test_quant_t_matches_transpose_then_quantize(R, NC):
    """The transposing weight quantisation equals quantising the transposed
    weight, with each weight's amax in its own slot."""
    torch.manual_seed(8)
    meta = F.Fp8Meta(DEV)
    ws = [(torch.randn(R, NC, device=DEV) * (i + 1) * 0.02).bfloat16() for i in range(3)]
    slots = [meta.slot(f"w{i}") for i in range(3)]
    for i, s in enumerate(slots):
        meta.scale[s] = 2.0 ** (6 - i)
    want = [F.quantize(w.t().contiguous(), meta, s, record=False) for w, s in zip(ws, slots)]
    got = [torch.empty(NC, R, dtype=F.FP8, device=DEV) for _ in ws]
    C().fp8_quant_t(ws, got, slots, meta.scale, meta.amax)
    for g, w in zip(got, want):
        assert torch.equal(g.view(torch.uint8), w.view(torch.uint8).view(NC, R))
    am = meta.amax_values()
    for w, s in zip(ws, slots):
        assert am[s].item() == w.float().abs().max().item()


def test_quant_colsum():
    """e5m2 quantisation fused with per-row-block column sums (input-projection
    bias gradients), strided input."""
    torch.manual_seed(9)
    gm = F.Fp8Meta(DEV, fmt=1)
    i = gm.slot("g")
    gm.scale[i] = 2.0 ** 10
    base = (torch.randn(1000, 3080, device=DEV) * 0.01).bfloat16()
    x = base[:, :3072]
    x8, part, nparts = F.quantize_colsum(x, gm, i, "test")
    want = F.quantize(x.contiguous(), gm, i, record=False).view(1000, 3072)
    assert torch.equal(x8.view(torch.uint8), want.view(torch.uint8))
    cs = part.view(nparts, 3072).sum(0)
    ref = x.float().sum(0)
    assert torch.allclose(cs, ref, rtol=1e-4, atol=1e-4)
    assert gm.amax_values()[i].item() == x.float().abs().max().item()


@pytest.mark.parametrize("causal,L,S,kv", [(True, 512, 512, True), (False, 300, 300, True),
                                            (False, 384, 200, False)])
def test_attn_bwd_emits_e5m2_grads(causal, L, S, kv):
    """The pipelined attention backward's e5m2 dQ (and dK / dV) equal
    quantising its bf16 gradients, amax recorded, bias-gradient partials sum
    to the column sums; skip_bf16 leaves the bf16 gradients untouched."""
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    torch.manual_seed(11)
    B, H, hd = 2, 3, 64
    q = torch.randn(B, L, H, hd, device=DEV).bfloat16()
    k, v = (torch.randn(B, S, H, hd, device=DEV).bfloat16() for _ in range(2))
    kv_len = torch.tensor([S, max(1, S - 37)], dtype=torch.int32, device=DEV)
    scale = hd ** -0.5
    o, lse = kk.attn_fwd(q, k, v, kv_len, scale, causal)
    do = torch.randn(B, L, H, hd, device=DEV).bfloat16()
    dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
    kk.attn_bwd(q, k, v, o, do, lse, dq, dk, dv, kv_len, scale, causal)
    gm = F.Fp8Meta(DEV, fmt=1)
    i = gm.slot("g")
    gm.scale[i] = 2.0 ** 12
    d = H * hd
    ncol = 3 * d if kv else d
    dq2 = torch.full_like(q, 7.0)
    dk2, dv2 = torch.full_like(k, 7.0), torch.full_like(v, 7.0)
    dq8 = torch.empty(q.shape, dtype=torch.float8_e5m2, device=DEV)
    dk8 = torch.empty(k.shape, dtype=torch.float8_e5m2, device=DEV) if kv else None
    dv8 = torch.empty(v.shape, dtype=torch.float8_e5m2, device=DEV) if kv else None
    part = torch.full((B * -(-L // 128) * ncol,), float("nan"), device=DEV)
    if not kv:  # skipping the bf16 dK / dV without their e5m2 copies would leave no output
        with pytest.raises(RuntimeError, match="skip_bf16 needs dk8"):
            kk.attn_bwd_g8(q, k, v, o, do, lse, dq2, dk2, dv2, kv_len, scale, causal, dq8, None,
                           None, gm.s(i), gm.a(i), part, ncol, 0, d, 2 * d, skip_bf16=True)
    np_ = kk.attn_bwd_g8(q, k, v, o, do, lse, dq2, dk2, dv2, kv_len, scale, causal, dq8, dk8, dv8,
                         gm.s(i), gm.a(i), part, ncol, 0, d, 2 * d)
    if kv:
        assert bool((dq2 == 7.0).all()) and bool((dk2 == 7.0).all())  # bf16 outputs skipped
    else:  # (default) the bf16 dK / dV are the output
        assert torch.equal(dk2, dk) and torch.equal(dv2, dv)

    def e5(x):
        return (x.float() * 2.0 ** 12).clamp(-57344, 57344).to(torch.float8_e5m2).view(torch.uint8)

    assert torch.equal(dq8.view(torch.uint8), e5(dq))
    cs = part[: np_ * ncol].view(np_, ncol).sum(0)
    assert torch.allclose(cs[:d], dq.float().sum((0, 1)).reshape(d), rtol=1e-3, atol=1e-3)
    am = dq.float().abs().max()
    if kv:
        assert torch.equal(dk8.view(torch.uint8), e5(dk))
        assert torch.equal(dv8.view(torch.uint8), e5(dv))
        assert torch.allclose(cs[d:2 * d], dk.float().sum((0, 1)).reshape(d), rtol=1e-3, atol=1e-3)
        assert torch.allclose(cs[2 * d:], dv.float().sum((0, 1)).reshape(d), rtol=1e-3, atol=1e-3)
        am = torch.maximum(am, torch.maximum(dk.float().abs().max(), dv.float().abs().max()))
    assert gm.amax_values()[i].item() == am.item()


def test_fused_fp8_adam_matches_separate_refresh(monkeypatch):
    """The Adam kernel that refreshes the e4m3 weight copies itself (scale
    update first, adam_chunk_kernel) trains bitwise like Adam followed by the
    scale update and the separate re-quantisation pass."""
    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.train import step as step_mod
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    cfg = model_config("tiny", src_vocab=96, tgt_vocab=96, dropout=0.1)
    data = SyntheticPairs(batch=16, src_len=16, tgt_len=17, src_vocab=96, tgt_vocab=96, seed=2)
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(step_mod, "FUSED_FP8_ADAM", fused)
        m = Transformer(cfg).build("cuda", seed=4)
        opt = Adam(m.store, cfg.d_model)
        st = F.Fp8State(m)
        if fused:
            assert st.weights.adam_chunks(m.store) is not None
        step = TrainStep(m, opt, None, workers=1.0, seed=3, fp8_state=st)
        for i in range(4):
            src, tgt = data.batch(i)
            step(src.cuda(), tgt.cuda())
        torch.cuda.synchronize()
        res[fused] = (m.store.flat.clone(), st.meta.scale.clone(),
                      torch.cat([w8.view(torch.uint8).reshape(-1) for _, w8, _, _ in st.weights.items]))
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)


def test_adam_chunk_kernel_matches_grid_adam_and_quant_multi():
    """adam_chunk_kernel on its own, against the grid-strided Adam kernel and
    fp8_quant_multi: a table with a ragged last chunk (< 4096), a range whose
    start is not a multiple of 4096, chunks refreshing two e4m3 copies (one
    starting mid-buffer, one of a length that is not a multiple of 4096) and
    plain chunks between them. p / m / v / the bf16 shadow must equal the
    grid kernel's bitwise, the e4m3 copies and their amax must equal
    fp8_quant_multi over the updated bf16 weights."""
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk

    torch.manual_seed(11)
    total = 3 * 4096 + 2052  # ragged tail
    p = torch.randn(total, device=DEV)
    g = torch.randn(total, device=DEV) * 0.1
    m0 = torch.randn(total, device=DEV) * 0.01
    v0 = torch.rand(total, device=DEV) * 0.01
    meta = F.Fp8Meta(DEV)
    w_a, w_b = (1000, 5000), (8192, 6148)  # (offset, numel) of two weights with e4m3 copies
    s_a, s_b = meta.slot("wa"), meta.slot("wb")
    meta.scale[s_a], meta.scale[s_b] = 64.0, 128.0
    y8a = torch.empty(w_a[1], dtype=F.FP8, device=DEV)
    y8b = torch.empty(w_b[1], dtype=F.FP8, device=DEV)
    rows = []
    pos = 4  # the whole-step range starts past 0 (not a multiple of 4096)

    def plain(a, b):
        for c0 in range(a, b, 4096):
            rows.append((c0, min(4096, b - c0), -1, 0))

    for (off, n), slot, y8 in ((w_a, s_a, y8a), (w_b, s_b, y8b)):
        plain(pos, off)
        for c0 in range(0, n, 4096):
            rows.append((off + c0, min(4096, n - c0), slot, y8.data_ptr() + c0))
        pos = off + n
    plain(pos, total)
    F.validate_chunk_table(rows, total, meta.scale.numel(), [(y8a.data_ptr(), y8a.numel()),
                                                               (y8b.data_ptr(), y8b.numel())])
    tab = torch.tensor(rows, dtype=torch.int64, device=DEV)
    args = (0.9, 0.98, 1e-9, 0.0, 512.0, 4000.0)

    def run(chunked):
        pp, gg, mm, vv = p.clone(), g.clone(), m0.clone(), v0.clone()
        sh = torch.zeros(total, dtype=torch.bfloat16, device=DEV)
        step = torch.tensor([7], dtype=torch.int64, device=DEV)
        if chunked:
            meta.amax.zero_()
            kk.adam_chunks(pp, gg, mm, vv, sh, tab, step, *args, 1.0, 0.0, 1, True, True,
                           meta.scale, meta.amax)
        else:
            sl = slice(4, total)
            kk.adam(pp[sl], gg[sl], mm[sl], vv[sl], sh[sl], step, *args, 1.0, 0.0, 1, True, True)
        torch.cuda.synchronize()
        return pp, gg, mm, vv, sh, step

    got, ref = run(True), run(False)
    for a, b, name in zip(got, ref, ("p", "g", "m", "v", "shadow", "step")):
        assert torch.equal(a, b), name
    sh = got[4]
    for (off, n), slot, y8 in ((w_a, s_a, y8a), (w_b, s_b, y8b)):
        want = F.quantize(sh[off:off + n], meta, slot, record=False)
        assert torch.equal(y8.view(torch.uint8), want.view(torch.uint8))
        assert meta.amax_values()[slot].item() == sh[off:off + n].float().abs().max().item()


@pytest.mark.parametrize("M,N,Kd", [(8192, 4096, 1024), (3000, 3072, 384), (8192, 1536, 256),
                                     (8192, 1040, 256), (1100, 1280, 256)])
def test_fp8_gemm_persistent_matches_oneshot(M, N, Kd):
    """The persistent 128x128 fp8 GEMM (fp8.hip gemm_fp8_pk_kernel: tiles
    walked by 2 workgroups per CU, the next tile's first K step in flight
    under the epilogue) writes bitwise what the one-shot grid writes: forward
    bias (+ReLU, e4m3 copy, amax) and the e5m2 dgrads (plain-weight transposing
    read; ReLU backward from the 8-bit mask with the fused column sums).
    Shapes with more tiles than two per CU (ragged M, a partial last column
    tile, the two-K-step minimum) take the persistent path; the last one
    stays one-shot."""
    from tensorflow_distributed_on_gke_amd.ops._ext import C as _C
    C = _C()
    torch.manual_seed(11)
    meta, gm = F.Fp8Meta(DEV), F.Fp8Meta(DEV, fmt=1)
    ia, ib, io = meta.slot("a"), meta.slot("b"), meta.slot("o")
    ig, igo = gm.slot("g"), gm.slot("go")
    meta.scale[io] = 8.0
    gm.scale[igo] = 256.0
    a8 = (torch.randn(M, Kd, device=DEV) * 4).to(F.FP8)
    b8 = (torch.randn(N, Kd, device=DEV) * 4).to(F.FP8)
    g8 = (torch.randn(M, Kd, device=DEV) * 4).to(F.BF8)
    w8 = (torch.randn(Kd, N, device=DEV) * 4).to(F.FP8)  # plain weight [out=K][in=N]
    bias = torch.randn(N, device=DEV)
    mask8 = torch.relu(torch.randn(M, N, device=DEV)).to(F.FP8)

    def run():
        outs = []
        y, y8 = F.gemm_fp8(a8, b8, bias, meta, ia, ib, relu=True, out8_slot=io, cfg=0)
        outs += [y, y8.view(torch.uint8)]
        y2, _ = F.gemm_fp8(a8, b8, bias, meta, ia, ib, cfg=0)
        outs.append(y2)
        d = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        d8 = F.gemm_bf8_dgrad(g8, gm, ig, w8, meta, ib, d, out8_slot=igo, cfg=0, w_plain=True)
        outs += [d, d8.view(torch.uint8)]
        cs = torch.zeros(N, device=DEV)
        r8 = F.gemm_bf8_dgrad(g8, gm, ig, w8, meta, ib, None,
                              out8_slot=igo, cfg=0, relu_aux8=mask8, colsum_out=cs, w_plain=True)
        outs += [r8.view(torch.uint8), cs]
        torch.cuda.synchronize()
        am = torch.cat([meta.amax_values()[io:io + 1], gm.amax_values()[igo:igo + 1]])
        return outs, am

    old = C.fp8_set_persist(0)
    try:
        ref, am_ref = run()
        meta.amax.zero_()
        gm.amax.zero_()
        C.fp8_set_persist(0xff)
        got, am_got = run()
    finally:
        C.fp8_set_persist(old)
    for i, (r, g) in enumerate(zip(ref, got)):
        assert torch.equal(r, g), (i, (r.float() - g.float()).abs().max().item())
    assert torch.equal(am_ref, am_got)
