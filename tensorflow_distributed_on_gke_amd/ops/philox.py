"""Host/CPU reference of the device dropout RNG (Philox4x32-10).

Bit-identical to `csrc/include/tdg_common.h`: the keep decision for element
`e` of a dropout site is the 16-bit half `e % 2` of word `(e % 8) // 2` of
Philox(counter=(e//8, offset), key=seed), kept iff >= rint(p * 2**16) (f32
arithmetic, as on the device), with offset = ctr * 4096 + site.
Used by the CPU reference ops so that CPU and GPU runs draw identical masks.
"""
from __future__ import annotations

import torch

_M0 = 0xD2511F53
_M1 = 0xCD9E8D57
_W0 = 0x9E3779B9
_W1 = 0xBB67AE85
_MASK = 0xFFFFFFFF


def _mulhilo(a: int | torch.Tensor, b: torch.Tensor):
    p = b * a  # int64 product of two uint32 fits in uint64; use int64 with masking
    # torch int64 overflow wraps (two's complement) -> low 32 bits are exact;
    # compute the high word via 16-bit limbs to avoid overflow.
    lo = p & _MASK
    b_lo = b & 0xFFFF
    b_hi = b >> 16
    a_lo = a & 0xFFFF
    a_hi = a >> 16
    t = a_lo * b_lo
    w0 = t & 0xFFFF
    k = t >> 16
    t = a_hi * b_lo + k
    w1 = t & 0xFFFF
    w2 = t >> 16
    t = a_lo * b_hi + w1
    k = t >> 16
    hi = a_hi * b_hi + w2 + k
    del w0
    return hi & _MASK, lo


def philox4x32(seed: int, offset: int, idx: torch.Tensor):
    """Return 4 uint32 words (as int64 tensors) for each counter index."""
    idx = idx.to(torch.int64)
    c0 = idx & _MASK
    c1 = (idx >> 32) & _MASK
    c2 = torch.full_like(idx, offset & _MASK)
    c3 = torch.full_like(idx, (offset >> 32) & _MASK)
    k0 = seed & _MASK
    k1 = (seed >> 32) & _MASK
    for _ in range(10):
        h0, l0 = _mulhilo(_M0, c0)
        h1, l1 = _mulhilo(_M1, c2)
        n0 = h1 ^ c1 ^ k0
        n2 = h0 ^ c3 ^ k1
        c0, c1, c2, c3 = n0, l1, n2, l0
        k0 = (k0 + _W0) & _MASK
        k1 = (k1 + _W1) & _MASK
    return c0, c1, c2, c3


def dropout_thresh(p: float) -> int:
    """rint(p * 2**16) in f32, clamped to 2**16 (tdg_common.h dropout_thresh)."""
    t = torch.tensor(p, dtype=torch.float32) * torch.tensor(65536.0, dtype=torch.float32)
    return int(min(65536.0, float(torch.round(t))))


def keep_mask(seed: int, offset: int, n: int, p: float) -> torch.Tensor:
    """Boolean keep mask for elements 0..n-1 of a dropout site."""
    thresh = dropout_thresh(p)
    groups = (n + 7) // 8
    w = philox4x32(seed, offset, torch.arange(groups, dtype=torch.int64))
    words = torch.stack(w, dim=1)  # [groups, 4]
    halves = torch.stack([words & 0xFFFF, words >> 16], dim=2).reshape(-1)[:n]
    return halves >= thresh


def rng_offset(ctr: int, site: int) -> int:
    return ctr * 4096 + site
