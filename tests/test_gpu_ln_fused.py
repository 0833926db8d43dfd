"""Post-LN block tails fused into the d_model-wide GEMMs (csrc/include/tdg_gemm_ln.h):
the forward LayerNorm in the output-projection / FFN2 epilogue and the
LayerNorm backward in the epilogue of the dgrad producing its input gradient,
with the row statistics exchanged between the 4 column tiles of a 128-row band.

Each is compared with the unfused kernels it replaces (the GEMM, then
ln_fwd / ln_bwd -- themselves tested against fp32 PyTorch in
test_gpu_kernels.py) and with an fp32 PyTorch reference of the same op; the
band counters must survive back-to-back launches and HIP-graph replays, and
a training run with the fusion must track the unfused one."""
import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import kernels as kk
from tensorflow_distributed_on_gke_amd.ops import philox

pytestmark = pytest.mark.gpu
DEV = "cuda"
D = 512


def _bf(t):
    return t.to(torch.bfloat16)


def _ref_fwd(a, w, b, x, gamma, beta, keep, p):
    s = _bf(a.float() @ w.float().t() + b).float()
    t = s * keep / (1 - p) if p > 0 else s
    h = _bf(x.float() + t).float()
    mu = h.mean(-1, keepdim=True)
    var = ((h - mu) ** 2).mean(-1, keepdim=True)
    rstd = torch.rsqrt(var + 1e-6)
    return (h - mu) * rstd * gamma + beta, h, mu.squeeze(1), rstd.squeeze(1)


def _keep(M, p, site, ctr):
    if p <= 0:
        return torch.ones(M, D, device=DEV)
    off = philox.rng_offset(int(ctr.item()), site)
    return philox.keep_mask(5, off, M * D, p).view(M, D).to(DEV).float()


@pytest.mark.parametrize("M,K,p", [(8192, 512, 0.1), (8192, 2048, 0.0), (1000, 512, 0.1), (256, 2048, 0.1)])
def test_gemm_ln_fwd_matches_unfused(M, K, p):
    torch.manual_seed(M + K)
    a = _bf(torch.randn(M, K, device=DEV))
    w = _bf(torch.randn(D, K, device=DEV) * K ** -0.5)
    b = torch.randn(D, device=DEV) * 0.1
    x = _bf(torch.randn(M, D, device=DEV))
    gamma = 1 + 0.1 * torch.randn(D, device=DEV)
    beta = 0.1 * torch.randn(D, device=DEV)
    ctr = torch.tensor([3], dtype=torch.int64, device=DEV)
    site = 17
    y, h, mean, rstd = kk.linear_ln_fwd(a, w, b, x, gamma, beta, p, 5, ctr, site, stages=3 if K <= 512 else 4)
    s = kk.linear_fwd(a, w, b)
    y0, h0, mean0, rstd0 = kk.ln_fwd(x, s, gamma, beta, p, 5, ctr, site)
    torch.cuda.synchronize()
    kk.ln_xch_check()
    # the sublayer output and h are bitwise the unfused ones (same bf16 s,
    # same dropout bits); the statistics differ only in summation order
    assert torch.equal(h, h0)
    assert torch.allclose(mean, mean0, rtol=1e-5, atol=1e-6)
    assert torch.allclose(rstd, rstd0, rtol=1e-4, atol=1e-6)
    assert (y.float() - y0.float()).abs().max().item() <= 2 * 2 ** -7 * y0.float().abs().max().item()
    ry, rh, rm, rr = _ref_fwd(a, w, b, x, gamma, beta, _keep(M, p, site, ctr), p)
    err = (y.float() - ry).norm() / ry.norm()
    assert err < 5e-3, err
    assert torch.allclose(rstd, rr, rtol=1e-3)


@pytest.mark.parametrize("M,K,with_c,p", [(8192, 1536, True, 0.1), (8192, 512, True, 0.0),
                                          (8192, 7010, False, 0.1), (1000, 2048, True, 0.1),
                                          (384, 6144, False, 0.0)])
def test_dgrad_ln_bwd_matches_unfused(M, K, with_c, p):
    torch.manual_seed(K + M)
    ld = (K + 63) // 64 * 64  # the vocabulary dgrad reads a padded dlogits row
    dY = _bf(torch.randn(M, ld, device=DEV) * 0.1)
    w = _bf(torch.randn(K, D, device=DEV) * K ** -0.5)
    c = _bf(torch.randn(M, D, device=DEV) * 0.1) if with_c else None
    h = _bf(torch.randn(M, D, device=DEV))
    mean = h.float().mean(-1)
    rstd = torch.rsqrt(h.float().var(-1, unbiased=False) + 1e-6)
    gamma = 1 + 0.1 * torch.randn(D, device=DEV)
    ctr = torch.tensor([2], dtype=torch.int64, device=DEV)
    site = 9
    outs = [torch.full((D,), 7.0, device=DEV) for _ in range(3)]
    defer = []
    dh, ds = kk.dgrad_ln_bwd(dY, w, c, h, mean, rstd, gamma, *outs, p, 5, ctr, site, defer,
                             stages=3 if K <= 512 else 4)
    kk.reduce_partials_multi(defer)
    # unfused: the dgrad (residual accumulated), then the LayerNorm backward
    dy = kk.linear_dgrad(dY, w, K, out=c.clone() if with_c else None,
                         beta=1.0 if with_c else 0.0)
    refs = [torch.full((D,), 7.0, device=DEV) for _ in range(3)]
    d2 = []
    dh0, ds0 = kk.ln_bwd(dy, h, mean, rstd, gamma, *refs, p, 5, ctr, site, defer=d2)
    kk.reduce_partials_multi(d2)
    torch.cuda.synchronize()
    kk.ln_xch_check()
    for got, want, name in ((dh, dh0, "dh"), (ds, ds0, "ds")):
        err = (got.float() - want.float()).norm() / want.float().norm()
        assert err < 2e-2, (name, err)
    for got, want, name in zip(outs, refs, ("dgamma", "dbeta", "dbias")):
        err = (got - want).norm() / want.norm()
        assert err < 1e-3, (name, err)
    # fp32 reference of the whole tail
    dyr = dY[:, :K].float() @ w.float() + (c.float() if with_c else 0)
    xh = (h.float() - mean[:, None]) * rstd[:, None]
    g = dyr * gamma
    dhr = rstd[:, None] * (g - g.mean(-1, keepdim=True) - xh * (g * xh).mean(-1, keepdim=True))
    keep = _keep(M, p, site, ctr)
    dsr = dhr * keep / (1 - p) if p > 0 else dhr
    assert (dh.float() - dhr).norm() / dhr.norm() < 2e-2
    assert (ds.float() - dsr).norm() / dsr.norm() < 2e-2
    assert (outs[0] - (dyr * xh).sum(0)).norm() / (dyr * xh).sum(0).norm() < 2e-2
    assert (outs[2] - dsr.sum(0)).norm() / dsr.sum(0).norm() < 2e-2


def test_band_counters_across_launches_and_graph_replays():
    """The arrival counters only grow: back-to-back launches, launches of
    different row counts and HIP-graph replays all meet at the right target
    (identical outputs every time, no spin timeout)."""
    torch.manual_seed(1)
    outs = {}
    for M in (8192, 640, 8192):
        a = _bf(torch.randn(M, 512, device=DEV))
        w = _bf(torch.randn(D, 512, device=DEV) * 0.05)
        b = torch.zeros(D, device=DEV)
        x = _bf(torch.randn(M, D, device=DEV))
        g1, b1 = torch.ones(D, device=DEV), torch.zeros(D, device=DEV)
        ys = [kk.linear_ln_fwd(a, w, b, x, g1, b1, 0.0, 0, None, 1)[0] for _ in range(3)]
        for y in ys[1:]:
            assert torch.equal(y, ys[0])
        outs.setdefault(M, ys[0])
    torch.cuda.synchronize()
    kk.ln_xch_check()
    M = 8192
    a = _bf(torch.randn(M, 512, device=DEV))
    w = _bf(torch.randn(D, 512, device=DEV) * 0.05)
    b = torch.zeros(D, device=DEV)
    x = _bf(torch.randn(M, D, device=DEV))
    g1, b1 = torch.ones(D, device=DEV), torch.zeros(D, device=DEV)
    ref = kk.linear_ln_fwd(a, w, b, x, g1, b1, 0.0, 0, None, 1)[0].clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        kk.linear_ln_fwd(a, w, b, x, g1, b1, 0.0, 0, None, 1)  # warm-up (workspaces)
        with torch.cuda.graph(graph):
            y_g = kk.linear_ln_fwd(a, w, b, x, g1, b1, 0.0, 0, None, 1)[0]
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(5):
        graph.replay()
        kk.linear_ln_fwd(a, w, b, x, g1, b1, 0.0, 0, None, 1)  # eager launches interleaved
    torch.cuda.synchronize()
    assert torch.equal(y_g, ref)
    kk.ln_xch_check()


@pytest.mark.parametrize("graph", [False, True])
def test_training_with_fused_layernorm_tracks_unfused(monkeypatch, graph):
    """Transformer-base layer shapes (d_model 512) with dropout: the fused
    tails (forward and backward) train like the separate LayerNorm kernels.
    One step's gradients -- every parameter, the LayerNorm / bias gradients
    folded from the fused partials included -- agree to bf16 noise, and the
    losses of four Adam steps track."""
    from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    monkeypatch.setattr(kk, "AUTOTUNE", False)
    cfg = model_config("tiny", d_model=512, heads=8, d_ff=2048, src_vocab=600, tgt_vocab=500,
                       dropout=0.1)
    data = SyntheticPairs(batch=16, src_len=64, tgt_len=65, src_vocab=600, tgt_vocab=500, seed=2)
    bs = [tuple(t.to(DEV) for t in data.batch(i)) for i in range(5)]
    res = {}
    for fused in ("0", "bwd", "all"):
        monkeypatch.setattr(kk, "LN_FUSED", fused)
        # gradients of one step (lr 0: Adam leaves the weights; the gradient
        # buffer keeps the step's gradients)
        m = Transformer(cfg).build(DEV, seed=4)
        step = TrainStep(m, Adam(m.store, cfg.d_model, lr=0.0), None, workers=1.0, seed=3)
        if graph:
            assert step.capture(*bs[0])
        step(*bs[1])
        grads = {p.name: p.grad.clone() for p in m.store.params}
        # losses of a short run
        m = Transformer(cfg).build(DEV, seed=4)
        step = TrainStep(m, Adam(m.store, cfg.d_model, lr=1e-3), None, workers=1.0, seed=3)
        if graph:
            assert step.capture(*bs[0])
        losses = [float(step(*b)[0]) for b in bs[1:]]
        torch.cuda.synchronize()
        res[fused] = (losses, grads)
    kk.ln_xch_check()
    l0, g0 = res["0"]
    for mode in ("bwd", "all"):
        l1, g1 = res[mode]
        for a, b in zip(l0, l1):
            assert abs(a - b) < 2e-3 * abs(a) + 1e-3, (mode, l0, l1)
        worst = max(((g1[k] - g0[k]).norm() / g0[k].norm().clamp_min(1e-12)).item() for k in g0)
        assert worst < 5e-2, (mode, worst)
        for k in g0:  # the fused LayerNorm's own parameters, folded from its partials
            if k.endswith(("/gamma", "/beta")):
                assert ((g1[k] - g0[k]).norm() / g0[k].norm()).item() < 3e-2, (mode, k)


@pytest.mark.parametrize("fwd", ["ln_fwd", "gemm_ln_fwd"])
def test_keep_bits_from_forward_match_regenerated_mask(fwd):
    """The forward's dropout keep bits (ln_fwd kbits, or the fused forward's)
    are the Philox mask bit for bit, and the fused backward reading them
    equals the one regenerating the mask."""
    torch.manual_seed(5)
    M, K, p, site = 8192, 512, 0.1, 21
    ctr = torch.tensor([4], dtype=torch.int64, device=DEV)
    a = _bf(torch.randn(M, K, device=DEV))
    w = _bf(torch.randn(D, K, device=DEV) * K ** -0.5)
    b = torch.zeros(D, device=DEV)
    x = _bf(torch.randn(M, D, device=DEV))
    g1, b1 = torch.ones(D, device=DEV), torch.zeros(D, device=DEV)
    kbits = torch.zeros(M, D // 8, dtype=torch.uint8, device=DEV)
    if fwd == "ln_fwd":
        s = kk.linear_fwd(a, w, b)
        _, h, mean, rstd = kk.ln_fwd(x, s, g1, b1, p, 5, ctr, site, kbits=kbits)
    else:
        _, h, mean, rstd = kk.linear_ln_fwd(a, w, b, x, g1, b1, p, 5, ctr, site, kbits=kbits)
    keep = _keep(M, p, site, ctr).bool()
    bits = torch.stack([(kbits.long() >> i) & 1 for i in range(8)], dim=-1).reshape(M, D).bool()
    assert torch.equal(bits, keep)
    dY = _bf(torch.randn(M, 1536, device=DEV) * 0.1)
    w2 = _bf(torch.randn(1536, D, device=DEV) * 0.03)
    c = _bf(torch.randn(M, D, device=DEV) * 0.1)
    outs = [[torch.zeros(D, device=DEV) for _ in range(3)] for _ in range(2)]
    r = []
    for i, kb in enumerate((None, kbits)):
        defer = []
        r.append(kk.dgrad_ln_bwd(dY, w2, c, h, mean, rstd, g1, *outs[i], p, 5, ctr, site, defer,
                                 kbits=kb))
        kk.reduce_partials_multi(defer)
    torch.cuda.synchronize()
    assert torch.equal(r[0][0], r[1][0]) and torch.equal(r[0][1], r[1][1])
    for a_, b_ in zip(outs[0], outs[1]):
        assert torch.equal(a_, b_)
    # the standalone LayerNorm backward reading the bits: bitwise the one
    # regenerating the mask
    dy = _bf(torch.randn(M, D, device=DEV) * 0.1)
    u = []
    for kb in (None, kbits):
        o3 = [torch.zeros(D, device=DEV) for _ in range(3)]
        dh, ds = kk.ln_bwd(dy, h, mean, rstd, g1, *o3, p, 5, ctr, site, kbits=kb)
        u.append((dh, ds, *o3))
    torch.cuda.synchronize()
    for a_, b_ in zip(*u):
        assert torch.equal(a_, b_)
