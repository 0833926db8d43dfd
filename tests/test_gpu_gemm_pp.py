"""Ping-pong 256x256 GEMM main loop (csrc/kernels/gemm.hip, gemm256_kernel
PP=true): numerics against an f32 PyTorch reference and BITWISE equality with
the lock-step loop (both issue every accumulator's MFMAs in the same k order),
over every layout / epilogue the 256x256 kernel serves, K from one K-tile (the
prologue / drain edge cases) up, and repeated launches (a staging race shows
up as run-to-run differences)."""
import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import kernels as kk
from tensorflow_distributed_on_gke_amd.ops._ext import C

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rand(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return ((torch.rand(*shape, generator=g) * 2 - 1) * scale)


def _bf(x):
    return x.to(torch.bfloat16).to(DEV)


@pytest.fixture
def pp_mode():
    old = C().get_gemm256_pp()
    yield lambda on: C().set_gemm256_pp(on)
    C().set_gemm256_pp(old)


def _both(pp_mode, fn):
    pp_mode(False)
    a = fn()
    pp_mode(True)
    b = fn()
    torch.cuda.synchronize()
    return a, b


def _close(a, ref, tol, what):
    err = (a.float().cpu() - ref.float().cpu()).abs().max().item()
    scale = ref.float().abs().max().item() + 1e-6
    assert err <= tol * scale, f"{what}: max err {err:.3e} vs {scale:.3e}"


@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (300, 520, 128), (512, 768, 192), (1024, 2048, 512),
                                   (8192, 1536, 512), (520, 264, 4096)])
@pytest.mark.parametrize("epi", ["bias_relu", "bias", "none"])
def test_pp_forward_nt(pp_mode, M, N, K, epi):
    x = _bf(_rand(M, K, seed=1))
    w = _bf(_rand(N, K, scale=0.5, seed=2))
    b = _rand(N, seed=3).to(DEV)
    e = {"bias_relu": kk.EPI_BIAS_RELU, "bias": kk.EPI_BIAS, "none": kk.EPI_NONE}[epi]

    def run():
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        kk.gemm(x, w, out, M, N, K, K, K, N, True, True, e, bias=b if e else None, cfg=(12, 1))
        return out

    a, p = _both(pp_mode, run)
    ref = x.float() @ w.float().t() + (b if e else 0)
    if e == kk.EPI_BIAS_RELU:
        ref = torch.relu(ref)
    _close(p, ref, 1e-2, "pp NT")
    assert torch.equal(a, p), "ping-pong and lock-step NT results differ"


@pytest.mark.parametrize("M,N,K", [(512, 128, 64), (300, 520, 192), (8192, 2048, 512)])
def test_pp_dgrad_nn_drelu(pp_mode, M, N, K):
    dy = _bf(_rand(M, K, seed=4))
    w = _bf(_rand(K, N, scale=0.5, seed=5))
    h = _bf(_rand(M, N, seed=6))

    def run():
        out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        kk.gemm(dy, w, out, M, N, K, K, N, N, True, False, kk.EPI_DRELU, aux=h, ldaux=N, cfg=(12, 1))
        return out

    a, p = _both(pp_mode, run)
    _close(p, (dy.float() @ w.float()) * (h.float() > 0), 1e-2, "pp NN drelu")
    assert torch.equal(a, p)


@pytest.mark.parametrize("M,N,K", [(512, 256, 64), (300, 520, 128), (2048, 512, 8192)])
@pytest.mark.parametrize("beta", [0.0, 1.0])
def test_pp_wgrad_tn(pp_mode, M, N, K, beta):
    ld = (M + 7) // 8 * 8
    a = _bf(_rand(K, ld, seed=24))
    x = _bf(_rand(K, N, seed=25))
    dw0 = _rand(M, N, seed=26).to(DEV)

    def run():
        dw = dw0.clone()
        C().gemm(a, x, dw, None, None, M, N, K, ld, N, N, 0, False, False, 0, 1.0, beta, 12, 1, None)
        return dw

    r, p = _both(pp_mode, run)
    _close(p, a[:, :M].float().t() @ x.float() + beta * dw0, 2e-3, "pp TN")
    assert torch.equal(r, p)


def test_pp_ragged_wgrad_repeatable(pp_mode):
    """The model's deferred weight gradients as one ragged launch (5 shapes,
    fused bias sums) at the training token count: equal to the lock-step loop
    bitwise, and bitwise stable over repeated launches."""
    T = 8192
    spec = [(1536, 512)] * 2 + [(512, 512)] * 3 + [(2048, 512)] * 2 + [(512, 2048)] * 2 + [(7010, 512)]
    dys, xs = [], []
    for i, (n_out, n_in) in enumerate(spec):
        ldy = 7040 if n_out == 7010 else n_out
        dy = _bf(_rand(T, ldy, seed=100 + i))
        dys.append(dy[:, :n_out] if n_out == 7010 else dy)
        xs.append(_bf(_rand(T, n_in, seed=200 + i)))

    def run():
        dws = [torch.zeros(n, k, dtype=torch.float32, device=DEV) for n, k in spec]
        bs = [torch.zeros(n, dtype=torch.float32, device=DEV) if i % 2 == 0 else None
              for i, (n, _) in enumerate(spec)]
        kk.wgrad_ragged(dys, xs, dws, beta=0.0, biases=bs)
        return dws, bs

    (lw, lb), (pw, pb) = _both(pp_mode, run)
    for i in range(len(spec)):
        assert torch.equal(lw[i], pw[i]), f"ragged problem {i} {spec[i]} differs"
        if lb[i] is not None:
            assert torch.equal(lb[i], pb[i])
    ref0 = dys[0].float().t() @ xs[0].float()
    _close(pw[0], ref0, 2e-3, "pp ragged[0]")
    _close(pw[-1], dys[-1].float().t() @ xs[-1].float(), 2e-3, "pp ragged vocab")
    pp_mode(True)
    for rep in range(4):
        w2, _ = run()
        torch.cuda.synchronize()
        for i in range(len(spec)):
            assert torch.equal(w2[i], pw[i]), f"repeat {rep}: problem {i} changed"
