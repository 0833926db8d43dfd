"""The deterministic CSR embedding backward (token sort, one wave per
vocabulary row or cut of a frequent row, fixed-point sums in registers,
embed.hip) against the fixed-point atomic kernel -- bitwise equal -- and
against a plain fp32 PyTorch index_add of the dropout-masked, scaled
gradient (reference: transformer_model.py:270-279, 301-308; the gradient of
Embedding -> * sqrt(d) -> + PE -> Dropout)."""
import math

import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import kernels as kk
from tensorflow_distributed_on_gke_amd.ops import philox

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _both(tok, dout, V, D, p, accumulate, init):
    ctr = torch.tensor([5], dtype=torch.int64, device=DEV)
    out = []
    for csr in (True, False):
        kk.EMBED_CSR = csr
        try:
            dt = init.clone()
            kk.embed_bwd(tok, dout, dt, math.sqrt(D), p, 99, ctr, 4, accumulate=accumulate)
            out.append(dt)
        finally:
            kk.EMBED_CSR = True
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize("D", [128, 256, 512, 1024])
@pytest.mark.parametrize("p", [0.0, 0.1])
@pytest.mark.parametrize("dist", ["uniform", "pad_heavy", "one_token"])
def test_embed_csr_matches_fixed_point(D, p, dist):
    B, L, V = 16, 73, 3001
    g = torch.Generator().manual_seed(D + int(p * 10))
    tok = torch.randint(0, V, (B, L), generator=g)
    if dist == "pad_heavy":  # right padding: one id with hundreds of rows (cut items)
        lens = torch.randint(5, L, (B,), generator=g)
        tok[torch.arange(L)[None, :] >= lens[:, None]] = 0
    elif dist == "one_token":
        tok[:] = 17
    dout = (torch.randn(B, L, D, generator=g) * 0.1).to(torch.bfloat16)
    init = torch.zeros(V, D, device=DEV)
    csr, fx = _both(tok.to(DEV), dout.to(DEV), V, D, p, False, init)
    assert torch.equal(csr, fx), "CSR and fixed-point atomic gradients differ"
    ks = (philox.keep_mask(99, philox.rng_offset(5, 4), B * L * D, p).view(B, L, D).float() / (1 - p)
          if p > 0 else torch.ones(B, L, D))
    ref = torch.zeros(V, D).index_add_(0, tok.view(-1), (dout.float() * ks * math.sqrt(D)).view(-1, D))
    err = (csr.cpu() - ref).abs().max().item()
    assert err <= 1e-4 * (ref.abs().max().item() + 1e-6), err


@pytest.mark.parametrize("tok_dtype", [torch.int32, torch.int64])
def test_embed_csr_accumulate_and_int32_tokens(tok_dtype):
    B, L, V, D = 8, 130, 7010, 512
    g = torch.Generator().manual_seed(3)
    tok = torch.randint(0, V, (B, L), generator=g)
    tok[:, 100:] = 0
    dout = (torch.randn(B, L, D, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    init = torch.randn(V, D, generator=g).to(DEV)
    csr, fx = _both(tok.to(tok_dtype).to(DEV), dout, V, D, 0.1, True, init)
    assert torch.equal(csr, fx)
    # repeated calls are bitwise stable (no stale workspace state)
    csr2, _ = _both(tok.to(tok_dtype).to(DEV), dout, V, D, 0.1, True, init)
    assert torch.equal(csr, csr2)


def test_embed_csr_transformer_shape():
    """The headline step's shape (8192 tokens, vocab 7765, d 512)."""
    B, L, V, D = 64, 128, 7765, 512
    g = torch.Generator().manual_seed(11)
    tok = torch.randint(1, V, (B, L), generator=g)
    lens = torch.randint(10, L + 1, (B,), generator=g)
    tok[torch.arange(L)[None, :] >= lens[:, None]] = 0
    dout = (torch.randn(B, L, D, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    csr, fx = _both(tok.to(DEV), dout, V, D, 0.1, False, torch.zeros(V, D, device=DEV))
    assert torch.equal(csr, fx)


@pytest.mark.parametrize("D", [512, 1024])
def test_embed_csr_forward_keep_bits(D):
    """The forward's keep bits (embed_fwd kbits) drive the CSR backward: the
    same gradient as regenerating the Philox mask, bitwise."""
    from tensorflow_distributed_on_gke_amd.models.transformer import positional_encoding

    B, L, V = 8, 100, 2000
    g = torch.Generator().manual_seed(D)
    tok = torch.randint(0, V, (B, L), generator=g)
    tok[:, 70:] = 0
    table = (torch.randn(V, D, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    pe = positional_encoding(128, D).to(DEV)
    ctr = torch.tensor([5], dtype=torch.int64, device=DEV)
    kb = torch.empty(B * L, D // 8, dtype=torch.uint8, device=DEV)
    out = kk.embed_fwd(tok.to(DEV), table, pe, math.sqrt(D), 0.1, 99, ctr, 4, kbits=kb)
    out0 = kk.embed_fwd(tok.to(DEV), table, pe, math.sqrt(D), 0.1, 99, ctr, 4)
    assert torch.equal(out, out0)
    keep = philox.keep_mask(99, philox.rng_offset(5, 4), B * L * D, 0.1).view(B * L, D)
    bits = torch.zeros(B * L, D // 8, dtype=torch.int64)
    for i in range(8):
        bits |= keep.view(B * L, D // 8, 8)[:, :, i].long() << i
    assert torch.equal(kb.cpu().long(), bits)
    dout = (torch.randn(B, L, D, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    a = torch.zeros(V, D, device=DEV)
    b = torch.zeros(V, D, device=DEV)
    kk.embed_bwd(tok.to(DEV), dout, a, math.sqrt(D), 0.1, 99, ctr, 4, kbits=kb)
    kk.embed_bwd(tok.to(DEV), dout, b, math.sqrt(D), 0.1, 99, ctr, 4)
    torch.cuda.synchronize()
    assert torch.equal(a, b)


def test_embed_csr_two_table_sort():
    """Both tables sorted by one launch (the training forward's form), each
    applied later: bitwise the fixed-point atomic gradients."""
    g = torch.Generator().manual_seed(21)
    D = 512
    ctr = torch.tensor([5], dtype=torch.int64, device=DEV)
    specs = [(7765, (64, 128)), (7010, (64, 127))]
    toks = []
    for V, (B, L) in specs:
        t = torch.randint(1, V, (B, L), generator=g)
        lens = torch.randint(5, L + 1, (B,), generator=g)
        t[torch.arange(L)[None, :] >= lens[:, None]] = 0
        toks.append(t.to(DEV))
    cs = kk.embed_csr_sort([(toks[0], specs[0][0], "t0"), (toks[1], specs[1][0], "t1")])
    for i, (V, (B, L)) in enumerate(specs):
        dout = (torch.randn(B, L, D, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
        a = torch.zeros(V, D, device=DEV)
        kk.embed_bwd(toks[i], dout, a, math.sqrt(D), 0.1, 99, ctr, 4, csr=cs[i])
        b = _both(toks[i], dout, V, D, 0.1, False, torch.zeros(V, D, device=DEV))[1]
        torch.cuda.synchronize()
        assert torch.equal(a, b), f"table {i}"
