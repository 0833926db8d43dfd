#!/usr/bin/env python3
"""L2 reuse model of the ragged weight-gradient launch (Transformer-base):
which 4 MiB operand panels (a 256-column slice of dY^T or X over all 8192
tokens) the tiles of each XCD round need, under the observed dispatch (block
b -> XCD b % 8, 32 concurrent tiles per XCD, xcd_remap'd tile order).
Assuming every round's tiles walk K in perfect step and share panels through
the XCD's L2, hit rate = 1 - unique panels / panel reads. Also the
compulsory panels of the launch (each read once chip-wide). Pure Python;
compare with the TCC_HIT / TCC_MISS table of profiles/r6/."""
import math

d, ff, L = 512, 2048, 6


def tiles(M, N):
    return math.ceil(M / 256), math.ceil(N / 256)


# shape runs in first-appearance (backward) order, as WgradQueue launches them
runs = [((7010, 512), 1), ((512, 2048), 2 * L), ((2048, 512), 2 * L), ((512, 512), 4 * L),
        ((1536, 512), 2 * L), ((2 * L * d, 512), 1)]
seq = []  # (problem, tm, tn) in ragged tile order
pid = 0
for (M, N), n in runs:
    for _ in range(n):
        tm_, tn_ = tiles(M, N)
        for t in range(tm_ * tn_):
            if tn_ <= tm_:
                tn, tm = t % tn_, t // tn_
            else:
                tm, tn = t % tm_, t // tm_
            seq.append((pid, tm, tn))
        pid += 1
T = len(seq)


def xcd_remap(bid, nwg):
    q, r = nwg // 8, nwg % 8
    x, i = bid % 8, bid // 8
    return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + i


per = [[] for _ in range(8)]
for b in range(T):
    per[b % 8].append(xcd_remap(b, T))
reads = uniq = 0
for x in range(8):
    for r0 in range(0, len(per[x]), 32):
        rnd = [seq[j] for j in per[x][r0:r0 + 32]]
        panels = {(p, "A", tm) for p, tm, _ in rnd} | {(p, "B", tn) for p, _, tn in rnd}
        reads += 2 * len(rnd)
        uniq += len(panels)
comp = len({(p, "A", tm) for p, tm, _ in seq} | {(p, "B", tn) for p, _, tn in seq})
print(f"tiles {T}; in-step model hit rate {1 - uniq / reads:.3f} ({uniq} panel loads of {reads} reads); "
      f"compulsory {comp} panels = {comp * 4 * 2 ** 20 // 128 / 1e6:.1f} M lines, ideal hit {1 - comp / reads:.3f}")
