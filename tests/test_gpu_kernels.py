"""Numerics of every gfx950 HIP kernel against a plain PyTorch f32 reference of
the same op (bf16-rounded inputs). Runs on the MI355X box (`-m gpu`)."""
import math

import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import kernels as kk
from tensorflow_distributed_on_gke_amd.ops import philox

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(*shape, generator=g) * 2 - 1) * scale


def _bf(x):
    return x.to(torch.bfloat16)


def _close(a, b, tol, what):
    a = a.float().cpu()
    b = b.float().cpu()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= tol * ref, f"{what}: max err {err:.3e} vs max |ref| {ref:.3e}"


# --------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (200, 136, 72), (1000, 7010, 128),
                                   (64, 64, 4096), (130, 520, 1000), (1024, 2048, 512), (300, 600, 192)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 12])
def test_gemm_forward_bias_relu(M, N, K, cfg):
    x = _bf(_rand(M, K, seed=1))
    w = _bf(_rand(N, K, scale=0.5, seed=2))
    b = _rand(N, seed=3)
    ref = torch.relu(x.float() @ w.float().t() + b)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    kk.gemm(x.to(DEV), w.to(DEV), out, M, N, K, K, K, N, True, True, kk.EPI_BIAS_RELU,
           bias=b.to(DEV), cfg=(cfg, 1))
    _close(out, ref, 1e-2, "gemm fwd")


def test_gemm_identity_asymmetric():
    # A = I with an asymmetric B catches transposed C writes
    n = 128
    a = torch.eye(n, dtype=torch.bfloat16)
    bmat = _bf(torch.arange(n * n, dtype=torch.float32).view(n, n) % 251)
    out = torch.empty(n, n, dtype=torch.float32, device=DEV)
    kk.gemm(a.to(DEV), bmat.to(DEV), out, n, n, n, n, n, n, True, True, kk.EPI_NONE, cfg=(0, 1))
    torch.testing.assert_close(out.cpu(), bmat.float().t())


@pytest.mark.parametrize("M,N,K", [(512, 128, 512), (300, 96, 200), (8192, 512, 2048), (1024, 2048, 512)])
@pytest.mark.parametrize("cfg", [0, 3, 12])
def test_gemm_dgrad_drelu(M, N, K, cfg):
    dy = _bf(_rand(M, N, seed=4))
    w = _bf(_rand(N, K, scale=0.5, seed=5))
    h = _bf(_rand(M, K, seed=6))
    ref = (dy.float() @ w.float()) * (h.float() > 0)
    out = torch.empty(M, K, dtype=torch.bfloat16, device=DEV)
    kk.gemm(dy.to(DEV), w.to(DEV), out, M, K, N, N, K, K, True, False, kk.EPI_DRELU, aux=h.to(DEV),
           ldaux=K, cfg=(cfg, 1))
    _close(out, ref, 1e-2, "gemm dgrad")


@pytest.mark.parametrize("M,N,K", [(1024, 512, 1536), (300, 200, 136), (130, 2048, 512)])
@pytest.mark.parametrize("cfg", [0, 1, 2, 4, 7, 8, 11])
def test_gemm_nn_epilogue_operands(M, N, K, cfg):
    """Every tile config of the NN (dgrad) kernel with an epilogue operand
    prefetched into registers before the main loop: beta*C residual
    accumulation, and the ReLU-backward mask."""
    dy = _bf(_rand(M, K, seed=31)).to(DEV)
    w = _bf(_rand(K, N, scale=0.5, seed=32)).to(DEV)
    c0 = _bf(_rand(M, N, seed=33)).to(DEV)
    out = c0.clone()
    kk.gemm(dy, w, out, M, N, K, K, N, N, True, False, kk.EPI_NONE, beta=1.0, cfg=(cfg, 1))
    _close(out, dy.float() @ w.float() + c0.float(), 1e-2, "gemm NN beta=1")
    h = _bf(_rand(M, N, seed=34)).to(DEV)
    kk.gemm(dy, w, out, M, N, K, K, N, N, True, False, kk.EPI_DRELU, aux=h, ldaux=N, cfg=(cfg, 1))
    _close(out, (dy.float() @ w.float()) * (h.float() > 0), 1e-2, "gemm NN drelu")


@pytest.mark.parametrize("M,N,K,splits", [(512, 128, 256, 1), (8192, 512, 512, 8), (1000, 7016, 64, 1),
                                          (4000, 200, 136, 3)])
def test_gemm_wgrad_f32(M, N, K, splits):
    # dW[N,K] = dy[M,N]^T x[M,K]  (A and B both M/N-contiguous)
    dy = _bf(_rand(M, N, seed=7))
    x = _bf(_rand(M, K, seed=8))
    ref = dy.float().t() @ x.float()
    out = torch.full((N, K), 3.0, dtype=torch.float32, device=DEV)
    ws = torch.empty(splits * N * K, dtype=torch.float32, device=DEV)
    K_ = K
    from tensorflow_distributed_on_gke_amd.ops._ext import C
    C().gemm(dy.to(DEV), x.to(DEV), out, None, None, N, K_, M, N, K_, K_, 0, False, False, 0, 1.0, 0.0,
             3, splits, ws if splits > 1 else None)
    _close(out, ref, 2e-3, "gemm wgrad")
    # beta accumulate
    C().gemm(dy.to(DEV), x.to(DEV), out, None, None, N, K_, M, N, K_, K_, 0, False, False, 0, 1.0, 1.0,
             0, 1, None)
    _close(out, 2 * ref, 2e-3, "gemm wgrad beta=1")


@pytest.mark.parametrize("M,N,K", [(512, 256, 1024), (300, 520, 128), (7010, 512, 256), (256, 264, 32)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
@pytest.mark.parametrize("cfg", [12, 20, 21, 22])
def test_gemm256_nn_tn(M, N, K, beta, cfg):
    """256x256 tiles (cfg 12) and the software-pipelined kernel (cfg 20-22:
    256x256 / 256x128 / 128x256, untracked fragment reads with counted waits)
    with MN-contiguous operands: dgrad NN (bf16, beta) and wgrad TN (f32,
    beta); NT with the bias + ReLU epilogue."""
    if cfg == 12 and K % 64:
        pytest.skip("256x256 lock-step tiles need K % 64 == 0 (falls back to cfg 0)")
    from tensorflow_distributed_on_gke_amd.ops._ext import C
    ld = (M + 7) // 8 * 8
    # NN: out[M,N] = dy[M,K] @ w[K,N]
    dy = _bf(_rand(M, K, seed=21)).to(DEV)
    w = _bf(_rand(K, N, scale=0.5, seed=22)).to(DEV)
    out = _bf(_rand(M, N, seed=23)).to(DEV)
    ref = dy.float() @ w.float() + beta * out.float()
    kk.gemm(dy, w, out, M, N, K, K, N, N, True, False, kk.EPI_NONE, beta=beta, cfg=(cfg, 1))
    _close(out, ref, 1e-2, "gemm256 NN")
    # TN: dw[M,N] = a[K,M]^T @ x[K,N]  (a stored [K][ld])
    a = _bf(_rand(K, ld, seed=24)).to(DEV)
    x = _bf(_rand(K, N, seed=25)).to(DEV)
    dw = _rand(M, N, seed=26).to(DEV)
    ref = a[:, :M].float().t() @ x.float() + beta * dw
    C().gemm(a, x, dw, None, None, M, N, K, ld, N, N, 0, False, False, 0, 1.0, beta, cfg, 1, None)
    _close(dw, ref, 2e-3, "gemm256 TN")
    # NT with the bias + ReLU epilogue (forward)
    xa = _bf(_rand(M, K, seed=27)).to(DEV)
    wt = _bf(_rand(N, K, scale=0.5, seed=28)).to(DEV)
    bias = _rand(N, seed=29).to(DEV)
    y = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ref = torch.relu(xa.float() @ wt.float().t() + bias)
    kk.gemm(xa, wt, y, M, N, K, K, K, N, True, True, kk.EPI_BIAS_RELU, bias=bias, cfg=(cfg, 1))
    _close(y, ref, 1e-2, "gemm256 NT bias relu")


@pytest.mark.parametrize("impl", [0, 1, 2])
def test_wgrad_ragged(impl, monkeypatch):
    """All deferred weight gradients of a model in ONE ragged 256x256 launch:
    5 shapes (incl. a padded-vocab operand, ld 7040 for 7010 rows), 17 problems.
    impl 0: lock-step loop; 1 / 2: pipelined loop at one wave per SIMD."""
    monkeypatch.setattr(kk, "WGRAD_IMPL", impl)
    T = 512
    spec = [(1536, 512)] * 3 + [(512, 512)] * 6 + [(2048, 512)] * 3 + [(512, 2048)] * 4 + [(7010, 512)]
    dys, xs, dws, refs = [], [], [], []
    for i, (n_out, n_in) in enumerate(spec):
        ldy = 7040 if n_out == 7010 else n_out
        dy = _bf(_rand(T, ldy, seed=100 + i)).to(DEV)
        x = _bf(_rand(T, n_in, seed=200 + i)).to(DEV)
        dw = _rand(n_out, n_in, seed=300 + i).to(DEV)
        refs.append(dy[:, :n_out].float().t() @ x.float() + dw)
        dys.append(dy[:, :n_out] if n_out == 7010 else dy)
        xs.append(x)
        dws.append(dw)
    # fused bias gradients on every other problem (row sums of dy^T over tokens)
    biases, brefs = [], []
    for i, (n_out, _) in enumerate(spec):
        if i % 2 == 0:
            b = _rand(n_out, seed=400 + i).to(DEV)
            brefs.append(dys[i].float().sum(0) + b)
            biases.append(b)
        else:
            biases.append(None)
            brefs.append(None)
    kk.wgrad_ragged(dys, xs, dws, beta=1.0, biases=biases)
    for i in range(len(spec)):
        _close(dws[i], refs[i], 2e-3, f"ragged wgrad {i} {spec[i]}")
        if brefs[i] is not None:
            _close(biases[i], brefs[i], 1e-4, f"ragged fused bias {i} {spec[i]}")


def test_linear_wrappers_padded_vocab():
    M, d, V, Vp = 300, 128, 7010, 7040
    x = _bf(_rand(M, d, seed=9)).to(DEV)
    w = _bf(_rand(V, d, scale=0.3, seed=10)).to(DEV)
    b = _rand(V, seed=11).to(DEV)
    lg = kk.linear_fwd(x, w, b, ldc=Vp)
    ref = x.float() @ w.float().t() + b
    _close(lg[:, :V], ref, 1e-2, "vocab fwd")
    dl = _bf(_rand(M, Vp, seed=12)).to(DEV)
    dl[:, V:] = 0
    dx = kk.linear_dgrad(dl, w, V)
    _close(dx, dl[:, :V].float() @ w.float(), 1e-2, "vocab dgrad")
    dw = torch.empty(V, d, dtype=torch.float32, device=DEV)
    kk.linear_wgrad(dl, x, V, dw)
    _close(dw, dl[:, :V].float().t() @ x.float(), 2e-3, "vocab wgrad")
    db = torch.empty(V, dtype=torch.float32, device=DEV)
    kk.colsum(dl, V, db)
    _close(db, dl[:, :V].float().sum(0), 1e-3, "colsum")


# --------------------------------------------------------------------------- attention
def _ref_attn(q, k, v, kv_len, causal, scale):
    q, k, v = q.float(), k.float(), v.float()
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    B, H, Lq, Lk = s.shape
    keys = torch.arange(Lk)
    mask = torch.zeros(B, 1, Lq, Lk, dtype=torch.bool)
    if kv_len is not None:
        mask |= (keys.view(1, 1, 1, Lk) >= kv_len.view(B, 1, 1, 1))
    if causal:
        mask |= (keys.view(1, Lk) > torch.arange(Lq).view(Lq, 1)).view(1, 1, Lq, Lk)
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, -1)
    return torch.einsum("bhqk,bkhd->bqhd", p, v), p


@pytest.mark.parametrize("hd", [16, 32, 64, 128])
@pytest.mark.parametrize("causal", [False, True])
@pytest.mark.parametrize("Lq,Lk", [(128, 128), (70, 200), (1, 33), (37, 100), (512, 512), (260, 390)])
def test_attention_fwd_bwd(hd, causal, Lq, Lk):
    if causal and Lq != Lk:
        pytest.skip("causal self-attention only")
    B, H = 3, 2
    torch.manual_seed(0)
    q = _bf(torch.randn(B, Lq, H, hd))
    k = _bf(torch.randn(B, Lk, H, hd))
    v = _bf(torch.randn(B, Lk, H, hd))
    kv_len = torch.tensor([Lk, max(1, Lk // 2), max(1, Lk - 5)], dtype=torch.int32)
    scale = 1 / math.sqrt(hd)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref, _ = _ref_attn(qr, kr, vr, kv_len, causal, scale)
    out, lse = kk.attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), kv_len.to(DEV), scale, causal)
    _close(out, ref.detach(), 2e-2, "attn fwd")
    dout = _bf(torch.randn(B, Lq, H, hd))
    ref.backward(dout.float())
    dq = torch.empty_like(q, device=DEV)
    dk = torch.empty_like(k, device=DEV)
    dv = torch.empty_like(v, device=DEV)
    kk.attn_bwd(q.to(DEV), k.to(DEV), v.to(DEV), out, dout.to(DEV), lse, dq, dk, dv, kv_len.to(DEV),
               scale, causal)
    _close(dv, vr.grad, 3e-2, "attn dv")
    _close(dk, kr.grad, 3e-2, "attn dk")
    _close(dq, qr.grad, 3e-2, "attn dq")


def _tf_attn(q, k, v, kv_len, causal, scale):
    """The reference's attention in fp32: -1e9 * mask added to the logits,
    padding and look-ahead masks combined by a maximum
    (transformer_model.py:94-108, 350-363)."""
    q, k, v = q.float(), k.float(), v.float()
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    B, H, Lq, Lk = s.shape
    keys = torch.arange(Lk)
    mask = (keys.view(1, 1, 1, Lk) >= kv_len.view(B, 1, 1, 1)).float().expand(B, 1, Lq, Lk)
    if causal:
        mask = torch.maximum(mask, (keys.view(1, Lk) > torch.arange(Lq).view(Lq, 1)).float().view(1, 1, Lq, Lk))
    p = torch.softmax(s + mask * -1e9, -1)
    return torch.einsum("bhqk,bkhd->bqhd", p, v), p


@pytest.mark.parametrize("causal,Lq,Lk,hd", [(False, 128, 128, 64), (True, 128, 128, 64), (False, 70, 100, 64),
                                             (False, 512, 512, 64), (True, 512, 512, 64), (False, 40, 33, 16)])
def test_attention_fully_masked_rows(causal, Lq, Lk, hd):
    """kv_len = 0 rows (an all-PAD sequence) follow the reference's fp32
    numerics: uniform attention over ALL keys (the look-ahead limit included
    in the mask), and TF's autograd through the mask add (dS from the uniform
    P, dQ / dK with the real scale). Short (fused backward) and long
    (dQ + dK/dV kernels) sequence paths, and the probabilities kernel."""
    B, H = 4, 2
    torch.manual_seed(3)
    q = _bf(torch.randn(B, Lq, H, hd))
    k = _bf(torch.randn(B, Lk, H, hd))
    v = _bf(torch.randn(B, Lk, H, hd))
    kv_len = torch.tensor([Lk, 0, max(1, Lk // 3), 0], dtype=torch.int32)
    scale = 1 / math.sqrt(hd)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref, pref = _tf_attn(qr, kr, vr, kv_len, causal, scale)
    out, lse = kk.attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), kv_len.to(DEV), scale, causal)
    _close(out, ref.detach(), 2e-2, "attn fwd (masked rows)")
    dout = _bf(torch.randn(B, Lq, H, hd))
    ref.backward(dout.float())
    dq, dk, dv = (torch.empty_like(t, device=DEV) for t in (q, k, v))
    kk.attn_bwd(q.to(DEV), k.to(DEV), v.to(DEV), out, dout.to(DEV), lse, dq, dk, dv, kv_len.to(DEV),
               scale, causal)
    _close(dv, vr.grad, 3e-2, "attn dv (masked rows)")
    _close(dk, kr.grad, 3e-2, "attn dk (masked rows)")
    _close(dq, qr.grad, 3e-2, "attn dq (masked rows)")
    if Lq <= 128:
        pr = kk.attn_probs(q.to(DEV), k.to(DEV), kv_len.to(DEV), scale, causal)
        _close(pr, pref.detach(), 1e-3, "probs (masked rows)")


@pytest.mark.parametrize("causal,Lq,Lk", [(False, 128, 128), (True, 128, 128), (False, 70, 100)])
def test_attention_bwd_more_items_than_cus(causal, Lq, Lk):
    """B*H = 267 (batch, head) items, more than the 256 CUs, ragged key lengths."""
    B, H, hd = 89, 3, 64
    torch.manual_seed(1)
    q = _bf(torch.randn(B, Lq, H, hd))
    k = _bf(torch.randn(B, Lk, H, hd))
    v = _bf(torch.randn(B, Lk, H, hd))
    kv_len = torch.randint(1, Lk + 1, (B,), dtype=torch.int32)
    kv_len[0] = Lk
    scale = 1 / math.sqrt(hd)
    qr, kr, vr = (t.float().requires_grad_() for t in (q, k, v))
    ref, _ = _ref_attn(qr, kr, vr, kv_len, causal, scale)
    out, lse = kk.attn_fwd(q.to(DEV), k.to(DEV), v.to(DEV), kv_len.to(DEV), scale, causal)
    dout = _bf(torch.randn(B, Lq, H, hd))
    ref.backward(dout.float())
    dq, dk, dv = (torch.empty_like(t, device=DEV) for t in (q, k, v))
    kk.attn_bwd(q.to(DEV), k.to(DEV), v.to(DEV), out, dout.to(DEV), lse, dq, dk, dv, kv_len.to(DEV),
               scale, causal)
    _close(dv, vr.grad, 3e-2, "attn dv")
    _close(dk, kr.grad, 3e-2, "attn dk")
    _close(dq, qr.grad, 3e-2, "attn dq")


def test_attention_strided_fused_qkv():
    # q/k/v as strided views into a fused [B, L, 3, H, hd] projection output
    B, L, H, hd = 2, 96, 8, 64
    qkv = _bf(torch.randn(B, L, 3, H, hd)).to(DEV)
    kv_len = torch.tensor([96, 50], dtype=torch.int32, device=DEV)
    out, _ = kk.attn_fwd(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2], kv_len, 0.125, True)
    c = qkv.cpu()
    ref, _ = _ref_attn(c[:, :, 0], c[:, :, 1], c[:, :, 2], kv_len.cpu(), True, 0.125)
    _close(out, ref, 2e-2, "strided attn")


def test_attention_probs():
    B, Lq, Lk, H, hd = 2, 10, 17, 2, 64
    q = _bf(torch.randn(B, Lq, H, hd))
    k = _bf(torch.randn(B, Lk, H, hd))
    kv_len = torch.tensor([17, 9], dtype=torch.int32)
    pr = kk.attn_probs(q.to(DEV), k.to(DEV), kv_len.to(DEV), 0.125, False)
    _, ref = _ref_attn(q, k, k, kv_len, False, 0.125)
    _close(pr, ref, 1e-3, "probs")


# --------------------------------------------------------------------------- layernorm
@pytest.mark.parametrize("D", [128, 512, 1024])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("rpb", [16, 32, 64])
def test_add_ln_fwd_bwd(D, p, rpb, monkeypatch):
    monkeypatch.setattr(kk, "LN_BWD_RPB", rpb)  # rows per backward workgroup
    M = 300
    seed, site = 1234, 7
    ctr = torch.tensor([5], dtype=torch.int64)
    x = _bf(torch.randn(M, D))
    s = _bf(torch.randn(M, D))
    gamma = torch.rand(D) + 0.5
    beta = torch.randn(D)
    y, h, mean, rstd = kk.ln_fwd(x.to(DEV), s.to(DEV), gamma.to(DEV), beta.to(DEV), p, seed,
                                ctr.to(DEV), site)
    keep = philox.keep_mask(seed, philox.rng_offset(5, site), M * D, p).view(M, D).float() if p > 0 else torch.ones(M, D)
    ks = keep / (1 - p)
    xr = x.float().requires_grad_()
    sr = s.float().requires_grad_()
    gr = gamma.clone().requires_grad_()
    br = beta.clone().requires_grad_()
    hr = xr + sr * ks
    ref = torch.nn.functional.layer_norm(hr, (D,), gr, br, 1e-6)
    _close(y, ref.detach(), 2e-2, "ln fwd")
    dy = _bf(torch.randn(M, D))
    ref.backward(dy.float())
    dg = torch.empty(D, device=DEV)
    db = torch.empty(D, device=DEV)
    dbias = torch.empty(D, device=DEV)
    dh, ds = kk.ln_bwd(dy.to(DEV), h, mean, rstd, gamma.to(DEV), dg, db, dbias, p, seed, ctr.to(DEV), site)
    _close(dh, xr.grad, 3e-2, "ln dh")
    _close(ds, sr.grad, 3e-2, "ln ds")
    _close(dg, gr.grad, 2e-2, "ln dgamma")
    _close(db, br.grad, 1e-2, "ln dbeta")
    _close(dbias, sr.grad.sum(0), 2e-2, "ln fused dbias")
    # deferred fold (partials kept per site, all folded in one launch later):
    # bitwise the same column sums, also when accumulating
    defer = []
    dg2, db2, dbias2 = (torch.full((D,), 2.0, device=DEV) for _ in range(3))
    kk.ln_bwd(dy.to(DEV), h, mean, rstd, gamma.to(DEV), dg2, db2, dbias2, p, seed, ctr.to(DEV),
              site, accumulate=True, defer=defer)
    assert len(defer) == 3 and torch.equal(dg2, torch.full((D,), 2.0, device=DEV))
    kk.reduce_partials_multi(defer)
    for got, want in ((dg2, dg), (db2, db), (dbias2, dbias)):
        torch.testing.assert_close(got, want + 2.0, rtol=0, atol=1e-5)


@pytest.mark.parametrize("N,off", [(512, 0), (512, 1), (100, 0), (36, 0)])
def test_reduce_partials_multi(N, off):
    """Deferred column folds: float4 strips (N % 4 == 0, 16-byte aligned) and
    the scalar kernel (misaligned output view, N % 4 != 0 not used by LN but
    N = 36 is a partial strip), plain and accumulating."""
    g = torch.Generator().manual_seed(N + off)
    items, want = [], []
    for i, P in enumerate((7, 130, 513)):
        part = torch.randn(P * N, generator=g).to(DEV)
        buf = torch.randn(N + off, generator=g).to(DEV)
        out = buf[off:]
        beta = 1.0 if i == 1 else 0.0
        want.append(part.view(P, N).double().sum(0).float() + (out.clone() if beta else 0))
        items.append((part, out, P, N, beta))
    kk.reduce_partials_multi(items)
    for (_, out, _, _, _), w in zip(items, want):
        torch.testing.assert_close(out, w, rtol=1e-5, atol=1e-4)


# --------------------------------------------------------------------------- embedding
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_embed_fwd_bwd(p):
    B, L, D, V = 4, 37, 128, 500
    from tensorflow_distributed_on_gke_amd.models.transformer import positional_encoding
    tok = torch.randint(0, V, (B, L))
    table = _bf(torch.randn(V, D) * 0.05)
    pe = positional_encoding(64, D)
    ctr = torch.tensor([3], dtype=torch.int64)
    out = kk.embed_fwd(tok.to(DEV), table.to(DEV), pe.to(DEV), math.sqrt(D), p, 77, ctr.to(DEV), 2)
    ks = (philox.keep_mask(77, philox.rng_offset(3, 2), B * L * D, p).view(B, L, D).float() / (1 - p)
          if p > 0 else torch.ones(B, L, D))
    ref = (table.float()[tok] * math.sqrt(D) + pe[:L]) * ks
    _close(out, ref, 1e-2, "embed fwd")
    dout = _bf(torch.randn(B, L, D))
    dt = torch.zeros(V, D, device=DEV)
    kk.embed_bwd(tok.to(DEV), dout.to(DEV), dt, math.sqrt(D), p, 77, ctr.to(DEV), 2)
    refg = torch.zeros(V, D).index_add_(0, tok.view(-1), (dout.float() * ks * math.sqrt(D)).view(-1, D))
    _close(dt, refg, 1e-4, "embed bwd")
    # deterministic path: bitwise identical across calls (and accumulate mode)
    dt2 = torch.full((V, D), 7.0, device=DEV)
    kk.embed_bwd(tok.to(DEV), dout.to(DEV), dt2, math.sqrt(D), p, 77, ctr.to(DEV), 2)
    assert torch.equal(dt, dt2)
    kk.embed_bwd(tok.to(DEV), dout.to(DEV), dt2, math.sqrt(D), p, 77, ctr.to(DEV), 2, accumulate=True)
    _close(dt2, 2 * refg, 1e-4, "embed bwd accumulate")


# --------------------------------------------------------------------------- cross-entropy
@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_xent(smoothing):
    M, V, Vp = 257, 7010, 7040
    lg = _bf(torch.randn(M, Vp) * 3)
    lab = torch.randint(1, V, (M,))
    lab[::7] = 0
    ntok = torch.zeros(1, device=DEV)
    lgd = lg.clone().to(DEV)
    kk.count_tokens(lab.to(DEV), ntok)
    rl = torch.empty(M, device=DEV)
    rc = torch.empty(M, device=DEV)
    kk.xent(lgd, V, lab.to(DEV), ntok, 2.0, smoothing, rl, rc, True)
    so = torch.empty(2, device=DEV)
    acc = torch.zeros(4, device=DEV)
    kk.xent_stats(rl, rc, ntok, 2.0, so, acc)
    x = lg.float()[:, :V].requires_grad_()
    mask = (lab != 0).float()
    n = mask.sum()
    logp = torch.log_softmax(x, -1)
    nll = -logp.gather(1, lab.view(-1, 1)).squeeze(1)
    row = ((1 - smoothing) * nll + smoothing * (-logp.mean(-1))) * mask
    loss = row.sum() / n / 2.0
    loss.backward()
    accr = ((x.argmax(-1) == lab).float() * mask).sum() / n
    assert ntok.item() == n.item()
    assert abs(so[0].item() - loss.item()) < 1e-3 * abs(loss.item())
    assert abs(so[1].item() - accr.item()) < 1e-6
    _close(lgd[:, :V], x.grad, 2e-2, "dlogits")
    assert lgd[:, V:].float().abs().max().item() == 0.0
    assert acc[2].item() == 1.0


# --------------------------------------------------------------------------- adam
def test_adam_keras_semantics():
    n = 4096
    p = torch.randn(n)
    g = torch.randn(n)
    m = torch.zeros(n)
    v = torch.zeros(n)
    pd, gd, md, vd = (t.clone().to(DEV) for t in (p, g, m, v))
    sh = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    step = torch.tensor([10], dtype=torch.int64, device=DEV)
    kk.adam(pd, gd, md, vd, sh, step, 0.9, 0.98, 1e-9, 0.0, 128.0, 4000.0)
    lr = 128 ** -0.5 * min(10 * 4000 ** -1.5, 10 ** -0.5)
    t = 11
    lr_t = lr * math.sqrt(1 - 0.98 ** t) / (1 - 0.9 ** t)
    m_ = g * 0.1
    v_ = g * g * 0.02
    ref = p - lr_t * m_ / (v_.sqrt() + 1e-9)
    _close(pd, ref, 1e-5, "adam p")
    _close(md, m_, 1e-6, "adam m")
    assert step.item() == 11
    assert gd.abs().max().item() == 0.0
    _close(sh, ref, 1e-2, "adam shadow")


# --------------------------------------------------------------------------- grouped launches
@pytest.mark.parametrize("G,M,N,Kd", [(5, 192, 128, 1000), (24, 512, 512, 2048), (3, 72, 2048, 333)])
def test_grouped_wgrad_and_colsum(G, M, N, Kd):
    """dW_i = dy_i^T x_i for G problems in one launch; bias grads grouped."""
    torch.manual_seed(0)
    dys = [_bf(torch.randn(Kd, M)).to(DEV) for _ in range(G)]
    xs = [_bf(torch.randn(Kd, N)).to(DEV) for _ in range(G)]
    dws = [torch.full((M, N), 3.0, device=DEV) for _ in range(G)]
    kk.wgrad_grouped(dys, xs, dws, beta=1.0)
    for i in range(G):
        ref = dys[i].float().t() @ xs[i].float() + 3.0
        _close(dws[i], ref, 1e-2, f"grouped wgrad {i}")
    outs = [torch.zeros(M, device=DEV) for _ in range(G)]
    kk.colsum_grouped(dys, outs)
    for i in range(G):
        _close(outs[i], dys[i].float().sum(0), 1e-3, f"grouped colsum {i}")


def test_gemm_beta_accumulate():
    """C += A B (bf16 out, the residual-gradient accumulation) vs fp32."""
    M, N, Kd = 512, 256, 384
    A = _bf(torch.randn(M, Kd)).to(DEV)
    B = _bf(torch.randn(Kd, N)).to(DEV)
    C0 = _bf(torch.randn(M, N)).to(DEV)
    ref = C0.float() + A.float() @ B.float()
    for cfg in ((8, 1), (13, 1), (6, 1)):
        C = C0.clone()
        kk.gemm(A, B, C, M, N, Kd, Kd, N, N, True, False, beta=1.0, cfg=cfg)
        _close(C, ref, 2e-2, f"beta=1 {cfg}")


@pytest.mark.parametrize("dtype", [torch.int64, torch.int32])
def test_prep_batch(dtype):
    """Fused batch preparation: teacher-forcing split, non-PAD lengths, label
    count and the RNG step bump, vs plain torch."""
    g = torch.Generator().manual_seed(5)
    B, S, T1 = 37, 71, 130
    src = torch.randint(1, 100, (B, S), generator=g, dtype=dtype)
    tgt = torch.randint(1, 100, (B, T1), generator=g, dtype=dtype)
    for b in range(B):  # right padding with PAD = 0
        src[b, torch.randint(1, S + 1, (1,), generator=g).item():] = 0
        tgt[b, torch.randint(2, T1 + 1, (1,), generator=g).item():] = 0
    ctr = torch.tensor([41], dtype=torch.int64, device=DEV)
    tgt_in, labels, sl, tl, ntok = kk.prep_batch(src.to(DEV), tgt.to(DEV), ctr)
    assert torch.equal(tgt_in.cpu(), tgt[:, :-1])
    assert torch.equal(labels.cpu(), tgt[:, 1:])
    assert torch.equal(sl.cpu(), (src != 0).sum(1).to(torch.int32))
    assert torch.equal(tl.cpu(), (tgt[:, :-1] != 0).sum(1).to(torch.int32))
    assert ntok.item() == float((tgt[:, 1:] != 0).sum())
    assert ctr.item() == 42
    assert kk.interior_pad_rows(reset=True) == 0  # right-padded only
    # a PAD inside a source row and one inside a target-input row are counted
    src[3, 2] = 0
    src[3, 5] = 7
    tgt[9, 1] = 0
    tgt[9, 4] = 7
    kk.prep_batch(src.to(DEV), tgt.to(DEV), ctr)
    assert kk.interior_pad_rows() == 2
    with pytest.raises(ValueError, match="right-padded"):
        kk.check_trailing_padding()
    assert kk.interior_pad_rows() == 0  # reset by the check


@pytest.mark.parametrize("cfg", [0, 4, 5, 6, 9, 10, 12, 13, 14, 20, 21, 22])
@pytest.mark.parametrize("relu", [False, True])
def test_linear_fwd_tile_configs(relu, cfg):
    """Every forward tile config of the table (the big preset's 256x128 /
    128x256 ones included) with the bias / bias+ReLU epilogue vs fp32, on
    ragged edges (M, N not tile multiples)."""
    M, N, K = 1000, 776, 512
    x = _bf(_rand(M, K, seed=71)).to(DEV)
    w = _bf(_rand(N, K, scale=1.0 / math.sqrt(K), seed=72)).to(DEV)
    b = _rand(N, scale=0.5, seed=73).to(DEV)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    epi = kk.EPI_BIAS_RELU if relu else kk.EPI_BIAS
    kk.gemm(x, w, out, M, N, K, K, K, N, True, True, epi, bias=b, cfg=(cfg, 1))
    ref = x.float() @ w.float().t() + b
    if relu:
        ref = torch.relu(ref)
    _close(out, ref, 1e-2, f"cfg{cfg} bias epilogue")


@pytest.mark.parametrize("cfg", [4, 5, 6, 9, 10, 13, 20, 21, 22])
def test_dgrad_tile_configs(cfg):
    """dgrad (NN: weight N-contiguous) for the tile configs the tuned table
    uses for d_model-wide outputs, with the beta = 1 accumulation."""
    M, N, K = 1000, 1024, 768
    dy = _bf(_rand(M, K, seed=81)).to(DEV)
    w = _bf(_rand(K, N, scale=1.0 / math.sqrt(K), seed=82)).to(DEV)
    c0 = _bf(_rand(M, N, seed=83)).to(DEV)
    out = c0.clone()
    kk.gemm(dy, w, out, M, N, K, K, N, N, True, False, kk.EPI_NONE, beta=1.0, cfg=(cfg, 1))
    ref = dy.float() @ w.float() + c0.float()
    _close(out, ref, 1e-2, f"cfg{cfg} dgrad beta=1")


@pytest.mark.parametrize("cfg", [20, 21, 22])
@pytest.mark.parametrize("K", [32, 64, 96])
def test_pipe_configs_short_k(cfg, K):
    """The LDS-DMA ring configs (gemm_pipe.h) with fewer K tiles than ring
    slots -- the one-K-tile case that faulted in the removed producer /
    consumer kernel sharing this prologue (docs/KERNELS.md): forward and
    beta = 1 dgrad vs fp32."""
    M, N = 520, 776
    x = _bf(_rand(M, K, seed=91)).to(DEV)
    w = _bf(_rand(N, K, scale=1.0 / math.sqrt(K), seed=92)).to(DEV)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    kk.gemm(x, w, out, M, N, K, K, K, N, True, True, kk.EPI_NONE, cfg=(cfg, 1))
    _close(out, x.float() @ w.float().t(), 1e-2, f"cfg{cfg} K={K} forward")
    wd = _bf(_rand(K, N, scale=1.0 / math.sqrt(K), seed=93)).to(DEV)
    c0 = _bf(_rand(M, N, seed=94)).to(DEV)
    out = c0.clone()
    kk.gemm(x, wd, out, M, N, K, K, N, N, True, False, kk.EPI_NONE, beta=1.0, cfg=(cfg, 1))
    _close(out, x.float() @ wd.float() + c0.float(), 1e-2, f"cfg{cfg} K={K} dgrad")


def test_no_library_gemm_in_training_step():
    """The training step runs only in-tree kernels: no hipBLASLt / rocBLAS
    (Cijk_* / rocblas_*) kernel in a profiled eager step of the base model,
    bf16 or fp8."""
    from torch.profiler import ProfilerActivity, profile

    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.ops.fp8 import Fp8State
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    for fp8 in (False, True):
        cfg = model_config("base")
        m = Transformer(cfg).build(DEV, seed=0)
        st = TrainStep(m, Adam(m.store, cfg.d_model), None, workers=1.0, seed=1,
                       fp8_state=Fp8State(m) if fp8 else None)
        data = SyntheticPairs(batch=16, src_len=64, tgt_len=65, src_vocab=cfg.src_vocab,
                              tgt_vocab=cfg.tgt_vocab, min_len=8)
        s, t = data.batch(0)
        st(s.to(DEV), t.to(DEV))
        torch.cuda.synchronize()
        with profile(activities=[ProfilerActivity.CUDA]) as prof:
            st(s.to(DEV), t.to(DEV))
            torch.cuda.synchronize()
        names = {e.name for e in prof.events() if e.device_type.name == "CUDA"}
        lib = sorted(n for n in names if n.startswith("Cijk") or "rocblas" in n.lower()
                     or "hipblaslt" in n.lower() or "Custom_Cijk" in n)
        assert not lib, f"library kernels in the step (fp8={fp8}): {lib[:5]}"
        assert any("gemm" in n for n in names), sorted(names)[:20]


def test_transpose_grouped_and_dgrad_t():
    """Grouped bf16 transpose (exact), and the relu-backward dgrad against the
    transposed weight copy equals the N-contiguous dgrad kernel's result to
    rounding (same math, different operand layout)."""
    ws = [_bf(_rand(512, 2048, scale=0.05, seed=80 + i)).to(DEV) for i in range(3)]
    wts = [torch.empty(2048, 512, dtype=torch.bfloat16, device=DEV) for _ in ws]
    kk.transpose_grouped(ws, wts)
    for w, wt in zip(ws, wts):
        assert torch.equal(wt, w.t())
    odd = _bf(_rand(136, 200, seed=90)).to(DEV)  # edge tiles
    odd_t = torch.empty(200, 136, dtype=torch.bfloat16, device=DEV)
    kk.transpose_grouped([odd], [odd_t])
    assert torch.equal(odd_t, odd.t())
    M = 1000
    dy = _bf(_rand(M, 512, seed=91)).to(DEV)
    h = _bf(_rand(M, 2048, seed=92)).to(DEV)
    a = kk.linear_dgrad_t(dy, wts[0], relu_aux=h)
    b = kk.linear_dgrad(dy, ws[0], 512, relu_aux=h)
    ref = (dy.float() @ ws[0].float()) * (h.float() > 0)
    _close(a, ref, 1e-2, "dgrad_t relu")
    _close(b, ref, 1e-2, "dgrad relu")
