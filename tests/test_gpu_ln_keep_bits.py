"""LayerNorm dropout keep bits: the training forward (ln_fwd kbits) saves the
Philox keep mask as 1 bit per element, and the LayerNorm backward reads it
instead of regenerating the mask. The bits must equal the Philox mask bit for
bit, and the backward reading them must be bitwise the one regenerating it.
(Reference: distributed_training_transformer/transformer_model.py:187-204 --
Dropout + residual + LayerNormalization of every post-LN block.)"""
import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import kernels as kk
from tensorflow_distributed_on_gke_amd.ops import philox

pytestmark = pytest.mark.gpu
DEV = "cuda"
D = 512


def _bf(t):
    return t.to(torch.bfloat16)


@pytest.mark.parametrize("M", [8192, 1000])
def test_keep_bits_from_forward_match_regenerated_mask(M):
    torch.manual_seed(5)
    K, p, site = 512, 0.1, 21
    ctr = torch.tensor([4], dtype=torch.int64, device=DEV)
    a = _bf(torch.randn(M, K, device=DEV))
    w = _bf(torch.randn(D, K, device=DEV) * K ** -0.5)
    b = torch.zeros(D, device=DEV)
    x = _bf(torch.randn(M, D, device=DEV))
    g1, b1 = torch.ones(D, device=DEV), torch.zeros(D, device=DEV)
    kbits = torch.zeros(M, D // 8, dtype=torch.uint8, device=DEV)
    s = kk.linear_fwd(a, w, b)
    _, h, mean, rstd = kk.ln_fwd(x, s, g1, b1, p, 5, ctr, site, kbits=kbits)
    off = philox.rng_offset(int(ctr.item()), site)
    keep = philox.keep_mask(5, off, M * D, p).view(M, D).to(DEV).bool()
    bits = torch.stack([(kbits.long() >> i) & 1 for i in range(8)], dim=-1).reshape(M, D).bool()
    assert torch.equal(bits, keep)
    dy = _bf(torch.randn(M, D, device=DEV) * 0.1)
    u = []
    for kb in (None, kbits):
        o3 = [torch.zeros(D, device=DEV) for _ in range(3)]
        dh, ds = kk.ln_bwd(dy, h, mean, rstd, g1, *o3, p, 5, ctr, site, kbits=kb)
        u.append((dh, ds, *o3))
    torch.cuda.synchronize()
    for a_, b_ in zip(*u):
        assert torch.equal(a_, b_)
