"""Fused block-level autograd ops of the encoder-decoder Transformer.

Every post-LN sublayer of the reference is ONE `torch.autograd.Function` with a
hand-written backward that sequences the gfx950 kernels and writes parameter
gradients straight into the flat f32 gradient buffer, notifying the
data-parallel engine as each becomes final (its bucket's all-reduce can start
while backward continues):

  SelfAttnBlockFn : y = LN(x + dropout(MHA(x, x, x)))          (encoder / decoder block 1)
  CrossAttnBlockFn: y = LN(x + dropout(MHA(enc, enc, x)))      (decoder block 2)
  FFNBlockFn      : y = LN(x + dropout(W2 relu(W1 x + b1) + b2))
  CrossKVFn       : K|V projections of the encoder output for ALL decoder
                    layers as one GEMM (N = layers*2*d)
  EmbedFn         : dropout(emb[tok] * sqrt(d) + PE)

Fusions this buys over per-op autograd: the residual gradient is added inside
the dgrad GEMM epilogue (beta = 1 onto the LayerNorm input gradient) instead
of an autograd add; the sublayer's output-bias gradient comes out of the
LayerNorm backward's column reduction; ReLU backward is the dgrad epilogue of
the second FFN GEMM; the encoder-output gradient of all cross attentions is
produced by one dgrad GEMM.

On CPU tensors the same ops run a plain-PyTorch f32 reference with identical
semantics (including the Philox dropout masks): the CPU test path and the
BASELINE "tiny on CPU" configuration. On GPU tensors only the HIP kernels run.

Reference semantics (distributed_training_transformer/transformer_model.py):
  MultiHeadAttention :112-166  (separate Q/K/V Dense; here fused [3d,d] / [L*2d,d])
  FFN                :169-175  (Dense(ff, relu) -> Dense(d))
  post-LN sublayer   :187-204, :219-248  (LN(x + dropout(sublayer(x))), eps 1e-6)
  embedding          :270-279, :301-308  (emb * sqrt(d) + PE, dropout)
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field
from typing import Optional

import torch

from tensorflow_distributed_on_gke_amd.models.params import Param, ParamStore
from tensorflow_distributed_on_gke_amd.ops import kernels as K
from tensorflow_distributed_on_gke_amd.ops import fp8, philox

LN_EPS = 1e-6
# deferred weight gradients as ragged 256x256-tile launches (else per-shape
# grouped launches of the tile table)
RAGGED_WGRAD = True


@dataclass
class RunCtx:
    """Per-forward runtime state shared by all layers."""

    training: bool = False
    dropout: float = 0.1
    seed: int = 0
    ctr: Optional[torch.Tensor] = None  # int64[1]: dropout stream counter (device-resident)
    accumulate: bool = False  # accumulate into existing grads (gradient accumulation)
    store: Optional[ParamStore] = None
    # inference probe: {site: [B,H,Lq,Lk] f32 attention weights} when set
    attn_maps: Optional[dict] = None
    # ops.fp8.Fp8State: FFN and attention-input forward GEMMs in e4m3 (BASELINE config 5)
    fp8: Optional[object] = None
    # WgradQueue: weight gradients deferred to the end of backward (grouped)
    wgrad: Optional["WgradQueue"] = None
    # {embedding site: ops.kernels.EmbCsr}: the token sorts of this forward's
    # embedding backwards (one launch for both tables, Transformer.features)
    emb_csr: Optional[dict] = None

    @property
    def p(self) -> float:
        return self.dropout if self.training else 0.0

    def cpu_offset(self, site: int) -> int:
        if self.ctr is None:
            return site
        return philox.rng_offset(int(self.ctr.item()), site)


@dataclass
class KVGrad:
    """Side channel collecting every decoder layer's d(K|V) into one buffer so
    the cross-K/V projection backward is a single GEMM pair. With the fp8
    attention backward on every decoder layer (`f8b`, decided by the forward
    of CrossKVFn), the layers write the e5m2 d(K|V) straight into `buf8` and
    their bias-gradient column sums into `part` ([B, layers * 2d]), and the
    bf16 K|V / d(K|V) are never materialised."""

    buf: Optional[torch.Tensor] = None
    dec_len: int = 0  # decoder sequence length of this forward (Transformer.decode)
    heads: int = 0
    f8b: bool = False
    buf8: Optional[torch.Tensor] = None
    part: Optional[torch.Tensor] = None
    wkv: Optional["Param"] = None  # the batched K|V projection (its e5m2 gradient slot)


def _dgrad_res(dy2: torch.Tensor, w: Param, N: int, dres: Optional[torch.Tensor]) -> torch.Tensor:
    """A block's input gradient dx = dy2 @ w (+ dres, the residual gradient
    already in dx: accumulated by the GEMM's beta = 1 epilogue)."""
    if dres is None:
        return K.linear_dgrad(dy2, w.compute, N)
    return _dgrad_into(dy2, w, N, dres)


def _keep_scale(rt: RunCtx, site: int, shape, device) -> Optional[torch.Tensor]:
    """CPU reference dropout multiplier (keep/(1-p)) drawn from the device RNG stream."""
    p = rt.p
    if p <= 0:
        return None
    n = math.prod(shape)
    keep = philox.keep_mask(rt.seed, rt.cpu_offset(site), n, p).view(shape)
    return keep.to(torch.float32).to(device) / (1.0 - p)


def _beta(rt: RunCtx) -> float:
    return 1.0 if rt.accumulate else 0.0


def _ready(rt: RunCtx, *params: Param) -> None:
    if rt.store is not None:
        for p in params:
            rt.store.grad_ready(p)


def _write_grad(p: Param, g: torch.Tensor, rt: RunCtx) -> None:
    if rt.accumulate:
        p.grad.add_(g.to(p.grad.dtype))
    else:
        p.grad.copy_(g.to(p.grad.dtype))


class WgradQueue:
    """Weight-gradient GEMMs deferred to the end of backward.

    Nothing in backward reads a weight gradient, so instead of one small
    long-K GEMM per layer (split-K slabs + a reduce kernel, 64x64 tiles to
    fill the chip) all of them run as ONE ragged launch of 256x256 whole-K
    tiles (ops.kernels.wgrad_ragged: 5 shapes, 62 problems, ~730 tiles for
    Transformer-base; bias gradients fused), or, with RAGGED_WGRAD = False, one
    grouped launch per shape (ops.kernels.wgrad_grouped) plus column sums.
    The data-parallel grad_ready notifications follow in backward order."""

    def __init__(self, flush_at_boundary: bool = False, wave_tiles: int = 0):
        self.items = []
        # data parallel: also flush when the decoder's backward is complete,
        # so the decoder-side buckets are all-reduced while the encoder's
        # backward runs (only without wave chunking)
        self.flush_at_boundary = flush_at_boundary
        # data parallel, ragged path: at every layer end launch as many whole
        # waves of `wave_tiles` tiles (one 256x256 whole-K tile per CU) as are
        # queued -- a launch of the queue's first n*wave_tiles tiles, cutting
        # the boundary problem by tile range -- so the all-reduce of those
        # gradients starts layers earlier while the launches together cost
        # exactly the waves of a single launch (chunks that each fill only
        # part of a wave cost a whole wave each: 4 chunks measured 1004 us vs
        # 745 us for one launch on Transformer-base)
        self.wave_tiles = wave_tiles
        # layer_end() calls per backward (set by the owner: encoder + decoder
        # layers). With wave chunking the LAST layer end flushes everything
        # queued, partial wave included: otherwise the remainder waits for the
        # end of backward and its gradients join the embedding gradients in
        # the final, fully exposed all-reduce span (71 MB at Transformer-base;
        # with the full flush the final span holds little more than the
        # source embedding)
        self.layers_per_step = 0
        self._layer_ends = 0
        self._cursor = 0  # tiles of items[0] already launched
        # deferred LayerNorm dgamma/dbeta/bias partial folds (one launch per flush)
        self.reductions = []
        self.reduced_params = []
        self.fp8_items = []
        self.small_per_shape = False

    def boundary(self) -> None:
        if self.flush_at_boundary and not self._chunking() and (self.items or self.reductions or self.fp8_items):
            self.flush()

    @staticmethod
    def _tiles(it) -> int:
        dy2, x2, N = it[0], it[1], it[2]
        return -(-N // 256) * -(-x2.shape[1] // 256)

    @staticmethod
    def _ragged_ok(it) -> bool:
        dy2, x2 = it[0], it[1]
        return x2.shape[0] % 64 == 0 and dy2.stride(0) % 8 == 0 and x2.stride(0) % 8 == 0

    def _chunking(self) -> bool:
        return bool(self.wave_tiles) and RAGGED_WGRAD

    def layer_end(self) -> None:
        """A decoder or encoder layer's backward is complete."""
        self._layer_ends += 1
        last = self.layers_per_step > 0 and self._layer_ends >= self.layers_per_step
        if self._chunking() and self.fp8_items:
            self._flush_fp8()  # (its gradients join the next all-reduce span)
        if not self._chunking() or not self.items:
            return
        if last or not all(self._ragged_ok(it) for it in self.items):
            self.flush()
            return
        queued = sum(self._tiles(it) for it in self.items) - self._cursor
        n = queued // self.wave_tiles * self.wave_tiles
        if n:
            self._launch_prefix(n)
            self._finish_flush()

    def add(self, dy2, x2, N, w: Param, b: Optional[Param], beta: float, rt: "RunCtx"):
        self.items.append((dy2, x2, N, w, b, beta, rt))

    def add_fp8(self, dy8, sa, x8, sb, w: Param, beta: float, rt: "RunCtx"):
        """An fp8 weight gradient (ops.fp8.wgrad_fp8), launched with the
        next flush / layer end as one ragged fp8 launch."""
        self.fp8_items.append((dy8, sa, x8, sb, w, beta, rt))

    def _flush_fp8(self) -> None:
        if not self.fp8_items:
            return
        by_beta = {}
        for it in self.fp8_items:
            by_beta.setdefault(it[5], []).append(it)
        for beta, its in by_beta.items():
            # equal shapes adjacent (one class each)
            its.sort(key=lambda it: (it[4].shape, it[0].stride(0), it[2].stride(0)))
            fp8.wgrad_fp8([it[0] for it in its], [it[1] for it in its], [it[2] for it in its],
                          [it[3] for it in its], [it[4].grad for it in its], beta)
        for it in self.fp8_items:
            _ready(it[6], it[4])
        self.fp8_items = []

    def step_done(self) -> None:
        """End of a backward: the layer-end count restarts."""
        self._layer_ends = 0

    def flush(self) -> None:
        self._flush_fp8()
        if self.items:
            # (small_per_shape: a flush of under half a wave of 256x256 tiles
            # -- the fp8 step's lone bf16 vocab projection -- runs per shape
            # on 128x128 tiles)
            if RAGGED_WGRAD and all(self._ragged_ok(it) for it in self.items) and (
                    not self.small_per_shape or self._cursor
                    or sum(self._tiles(it) for it in self.items) >= K.NUM_CU // 2):
                self._launch_prefix(sum(self._tiles(it) for it in self.items) - self._cursor)
            else:  # (never partially launched: chunking needs the ragged path)
                self._flush_grouped()
                self._flush_bias()
                self._done = self.items
                self.items = []
        else:
            self._done = []
        self._finish_flush()

    def _finish_flush(self) -> None:
        if self.reductions:
            K.reduce_partials_multi(self.reductions)
        done = getattr(self, "_done", [])
        for dy2, x2, N, w, b, beta, rt in done:
            _ready(rt, w, *([b] if b is not None else []))
        for rt, p in self.reduced_params:
            _ready(rt, p)
        rts = [it[6] for it in done] + [rp[0] for rp in self.reduced_params]
        if rts and rts[0].store is not None:
            rts[0].store.grad_sync()
        self._done = []
        self.reductions = []
        self.reduced_params = []

    def _launch_prefix(self, n: int) -> None:
        """Launch the first n not-yet-launched tiles of the queue (whole-K
        256x256 tiles, bias gradients fused): the items they complete move to
        self._done; a cut item stays at the queue head with self._cursor set."""
        sel = []  # (item, t_first, t_count)
        done = []
        left = n
        while left > 0 and self.items:
            it = self.items[0]
            avail = self._tiles(it) - self._cursor
            take = min(avail, left)
            sel.append((it, self._cursor, take))
            left -= take
            if take == avail:
                done.append(self.items.pop(0))
                self._cursor = 0
            else:
                self._cursor += take
        self._done = done
        # one launch per (token count, beta); within it full problems of equal
        # shape adjacent (one class each), cut problems as classes of their own
        runs = {}
        for it, first, cnt in sel:
            dy2, x2, N, w, b, beta, rt = it
            full = first == 0 and cnt == self._tiles(it)
            key = (N, x2.shape[1], dy2.stride(0), x2.stride(0)) if full else ("cut", id(it), first)
            runs.setdefault((x2.shape[0], beta), {}).setdefault(key, []).append((it, first, cnt))
        for (_, beta), by_shape in runs.items():
            groups = list(by_shape.values())
            for s0 in range(0, len(groups), K.RAGGED_MAX_SHAPES):
                chunk = [e for grp in groups[s0:s0 + K.RAGGED_MAX_SHAPES] for e in grp]
                for c0 in range(0, len(chunk), K.RAGGED_MAX_PROBLEMS):
                    part = chunk[c0:c0 + K.RAGGED_MAX_PROBLEMS]
                    K.wgrad_ragged([e[0][0] for e in part], [e[0][1] for e in part],
                                   [e[0][3].grad for e in part], beta,
                                   [e[0][4].grad if e[0][4] is not None else None for e in part],
                                   ranges=[(e[1], e[2]) for e in part])

    def _flush_grouped(self) -> None:
        groups = {}
        for it in self.items:
            dy2, x2, N, w, b, beta, rt = it
            key = (tuple(dy2.shape), dy2.stride(0), tuple(x2.shape), x2.stride(0), N, beta)
            groups.setdefault(key, []).append(it)
        for key, items in groups.items():
            for c0 in range(0, len(items), 32):
                chunk = items[c0:c0 + 32]
                beta = chunk[0][5]
                if len(chunk) == 1:
                    dy2, x2, N, w, *_ = chunk[0]
                    K.linear_wgrad(dy2, x2, N, w.grad, beta)
                else:
                    K.wgrad_grouped([i[0] for i in chunk], [i[1] for i in chunk],
                                    [i[3].grad for i in chunk], beta)

    def _flush_bias(self) -> None:
        bgroups = {}
        for dy2, x2, N, w, b, beta, rt in self.items:
            if b is not None:
                bgroups.setdefault((tuple(dy2.shape), dy2.stride(0), N, beta), []).append((dy2, b))
        for (shape, ld, N, beta), items in bgroups.items():
            for c0 in range(0, len(items), 32):
                chunk = items[c0:c0 + 32]
                if len(chunk) == 1:
                    K.colsum(chunk[0][0], N, chunk[0][1].grad, beta)
                else:
                    K.colsum_grouped([i[0] for i in chunk], [i[1].grad for i in chunk], beta)


def _wgrad(rt: RunCtx, dy2, x2, N: int, w: Param, b: Optional[Param] = None) -> None:
    """dW (+ bias grad) of a Linear on the GPU: deferred (rt.wgrad) or now."""
    bt = _beta(rt)
    if rt.wgrad is not None:
        rt.wgrad.add(dy2, x2, N, w, b, bt, rt)
        return
    K.linear_wgrad(dy2, x2, N, w.grad, bt)
    if b is not None:
        K.colsum(dy2, N, b.grad, bt)
    _ready(rt, w, *([b] if b is not None else []))


def _attn_lean(rt: RunCtx, M: int, w_in: Param, w_out: Optional[Param], d: int) -> bool:
    """Attention block with fp8 projections in forward and backward (fp8
    state with ATTN_PROJ_FP8; weight gradients through the deferred queue)."""
    st = rt.fp8
    return (st is not None and rt.training and rt.wgrad is not None and fp8.ATTN_PROJ_FP8
            and id(w_in) in st.proj_bwd and (w_out is None or id(w_out) in st.attn_out)
            and fp8.wgrad_fp8_ok(M, d, d))


def _fp8_grad_bias(g: torch.Tensor, g_slot: int, b: Param, rt: RunCtx, key: str):
    """e5m2 copy of the bf16 gradient g [M, N] and, from the same pass, the
    bias gradient (column sums) -- folded with the queue's other deferred
    column reductions at the next flush (one launch)."""
    st = rt.fp8
    g8, part, nparts = fp8.quantize_colsum(g, st.gmeta, g_slot, key)
    q = rt.wgrad
    q.reductions.append((part, b.grad, nparts, g.shape[1], _beta(rt)))
    q.reduced_params.append((rt, b))
    return g8


def _fold_bias_later(rt: RunCtx, part: torch.Tensor, nparts: int, N: int, b: Param) -> None:
    """b's gradient = column sums of the [nparts, N] partials, folded with the
    queue's other deferred column reductions at the next flush."""
    q = rt.wgrad
    q.reductions.append((part, b.grad, nparts, N, _beta(rt)))
    q.reduced_params.append((rt, b))


def _fp8_dgrad_into(g8, g_slot: int, w: Param, out: torch.Tensor, rt: RunCtx, beta: float) -> None:
    """out (=|+= beta) dequant(g8 (e5m2) @ w) against w's e4m3 copy (read
    N-contiguous by the kernel, fp8.DGRAD_PLAIN_W; else its transposed copy)."""
    st = rt.fp8
    wt8, swt = st.weights.get(w, transposed=not fp8.DGRAD_PLAIN_W)
    fp8.gemm_bf8_dgrad(g8, st.gmeta, g_slot, wt8, st.meta, swt, out, beta=beta,
                       w_plain=fp8.DGRAD_PLAIN_W)


def _fp8_dgrad8(g8, g_slot: int, w: Param, out_slot: int, rt: RunCtx) -> torch.Tensor:
    """e5m2 copy only (no bf16 output) of dequant(g8 (e5m2) @ w) in the
    gradient slot out_slot (amax recorded): the fp8 attention backward's dO."""
    st = rt.fp8
    wt8, swt = st.weights.get(w, transposed=not fp8.DGRAD_PLAIN_W)
    return fp8.gemm_bf8_dgrad(g8, st.gmeta, g_slot, wt8, st.meta, swt, None, out8_slot=out_slot,
                              w_plain=fp8.DGRAD_PLAIN_W)


def _f8_bwd_planned(rt: RunCtx, lean: bool, Lq: int, Lk: int, hd: int) -> bool:
    """Forward-time decision: will this (e4m3-forward) attention block's
    backward run on the fp8 kernel? Then the bf16 copies of its projection
    outputs are never read and not written. (Not with attention maps: they
    read the bf16 Q / K.)"""
    return (lean and fp8.ATTN_BWD_F8 and rt.attn_maps is None and K.attn_bwd_f8_ok(Lq, Lk, hd))


def _attn_f8_bwd(ctx, Lq: int, Lk: int, hd: int) -> bool:
    """Does this attention block's fp8 backward run on the fp8 kernel (its
    forward decided so: _f8_bwd_planned, and kept the e4m3 operands)?"""
    return getattr(ctx, "f8b", False) and getattr(ctx, "q8", None) is not None


# =============================================================================== LN helpers
def _proj_ln_fwd(a2, w: Param, b: Param, x, gamma: Param, beta: Param, site: int, rt: RunCtx):
    """GPU block tail y = LN(x + dropout(a2 @ w^T + b)) -> (y, saved): the
    output-projection GEMM (bias fused) then the fused dropout + residual +
    LayerNorm kernel. (GEMM + LayerNorm in one launch measured slower on
    MI355X, both as full-row tiles -- every workgroup streams all of W,
    csrc/lab/gemm_ln.hip -- and as 128-column tiles exchanging row partials
    across workgroups: profiles/r5/ln_fused_ab.txt.)"""
    s = K.linear_fwd(a2, w.compute, b.master)
    return _ln_fwd(x, s.view(x.shape), gamma, beta, site, rt)


# the training forward's LayerNorms save their dropout keep bits (1 bit per
# element) for the backward, which reads them instead of regenerating the
# Philox mask (ln_bwd kbits)
LN_KEEP_BITS = os.environ.get("TDG_LN_KEEP_BITS", "1") != "0"


def _kbits(rt: RunCtx, x: torch.Tensor) -> Optional[torch.Tensor]:
    """Keep-bit bitmap [M, D / 8] of a training LayerNorm with dropout."""
    D = x.shape[-1]
    if LN_KEEP_BITS and x.is_cuda and rt.training and rt.p > 0 and D % 512 == 0:
        return torch.empty(x.numel() // D, D // 8, dtype=torch.uint8, device=x.device)
    return None


def _ln_fwd(x, s, gamma: Param, beta: Param, site: int, rt: RunCtx):
    """Returns (y, saved) for y = LN(x + dropout(s)); saved = (h, mean, rstd,
    CPU keep scale, GPU keep bits)."""
    if x.is_cuda:
        y8 = s8 = a8 = None
        slot = rt.fp8.ln_slots.get(id(gamma)) if rt.fp8 is not None else None
        if slot is not None:  # this LN feeds an fp8 GEMM: emit its e4m3 copy too
            y8 = torch.empty(x.shape, dtype=fp8.FP8, device=x.device)
            s8, a8 = rt.fp8.meta.s(slot), rt.fp8.meta.a(slot)
            rt.fp8.stash[slot] = y8
        kbits = _kbits(rt, x)
        y, h, mean, rstd = K.ln_fwd(x.contiguous(), s.contiguous(), gamma.master, beta.master,
                                    rt.p, rt.seed, rt.ctr, site, y8=y8, s8=s8, amax8=a8, kbits=kbits)
        return y, (h, mean, rstd, None, kbits)
    ks = _keep_scale(rt, site, s.shape, s.device)
    h = x + (s * ks if ks is not None else s)
    mean = h.mean(-1, keepdim=True)
    rstd = torch.rsqrt(((h - mean) ** 2).mean(-1, keepdim=True) + LN_EPS)
    return (h - mean) * rstd * gamma.master + beta.master, (h, mean, rstd, ks, None)


def _ln_bwd(dy, saved, gamma: Param, beta: Param, sub_bias: Param, site: int, rt: RunCtx,
            ds8_slot: Optional[int] = None):
    """Returns (dh, ds): dh = dL/d(residual input) (fresh, writable), ds =
    dL/d(sublayer output). Also writes dgamma, dbeta and the sublayer's output
    bias gradient (sum of ds over rows). ds8_slot (GPU, fp8 backward): ds is
    returned as its e5m2 copy only (scale slot ds8_slot of rt.fp8.gmeta,
    amax recorded), the bf16 ds is not written."""
    h, mean, rstd, ks = saved[:4]
    if dy.is_cuda:
        q = rt.wgrad
        ds8 = s8 = a8 = None
        if ds8_slot is not None:
            gm = rt.fp8.gmeta
            ds8 = torch.empty(dy.shape, dtype=gm.dtype, device=dy.device)
            s8, a8 = gm.s(ds8_slot), gm.a(ds8_slot)
        dh, ds = K.ln_bwd(dy.contiguous(), h, mean, rstd, gamma.master, gamma.grad, beta.grad,
                          sub_bias.grad, rt.p, rt.seed, rt.ctr, site, want_ds=ds8 is None,
                          accumulate=rt.accumulate, defer=q.reductions if q is not None else None,
                          ds8=ds8, s8=s8, amax8=a8, kbits=saved[4])
        if ds8 is not None:
            ds = ds8
        if q is not None:  # folded (and reported ready) with the next wgrad flush
            q.reduced_params += [(rt, gamma), (rt, beta), (rt, sub_bias)]
            return dh, ds
    else:
        xhat = (h - mean) * rstd
        D = h.shape[-1]
        g = dy * gamma.master
        dh = rstd * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).mean(-1, keepdim=True))
        ds = dh * ks if ks is not None else dh
        _write_grad(gamma, (dy * xhat).reshape(-1, D).sum(0), rt)
        _write_grad(beta, dy.reshape(-1, D).sum(0), rt)
        _write_grad(sub_bias, ds.reshape(-1, D).sum(0), rt)
    _ready(rt, gamma, beta, sub_bias)
    return dh, ds


def _dgrad_into(dy2: torch.Tensor, w: Param, N: int, dx: torch.Tensor) -> torch.Tensor:
    """dx += dy2 @ w (the residual gradient already sits in dx)."""
    if dy2.is_cuda:
        return K.linear_dgrad(dy2, w.compute, N, out=dx.view(dy2.shape[0], -1), beta=1.0)
    dx.view(dy2.shape[0], -1).add_(dy2 @ w.master)
    return dx


# =============================================================================== embedding
class EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, tok, table: Param, pe: torch.Tensor, site: int, rt: RunCtx):
        d = table.shape[1]
        scale = math.sqrt(d)
        ctx.table, ctx.site, ctx.rt, ctx.scale = table, site, rt, scale
        ctx.save_for_backward(tok)
        if tok.is_cuda:
            # training with dropout: the keep bits for the CSR backward
            ctx.kbits = None
            ctx.csr = rt.emb_csr.get(site) if rt.emb_csr else None
            if ctx.csr is not None and rt.p > 0 and d % 512 == 0:
                ctx.kbits = torch.empty(tok.numel(), d // 8, dtype=torch.uint8, device=tok.device)
            return K.embed_fwd(tok, table.compute, pe, scale, rt.p, rt.seed, rt.ctr, site,
                               kbits=ctx.kbits)
        B, L = tok.shape
        x = table.master[tok] * scale + pe[:L].unsqueeze(0)
        ks = _keep_scale(rt, site, x.shape, x.device)
        ctx.ks = ks
        return x * ks if ks is not None else x

    @staticmethod
    def backward(ctx, dout):
        (tok,) = ctx.saved_tensors
        table, rt = ctx.table, ctx.rt
        if dout.is_cuda:
            dc = dout.contiguous()
            K.embed_bwd(tok, dc, table.grad, ctx.scale, rt.p, rt.seed, rt.ctr, ctx.site,
                        accumulate=rt.accumulate, kbits=ctx.kbits, csr=ctx.csr)
            _ready(rt, table)
            return None, None, None, None, None, None
        else:
            g = dout * ctx.ks if ctx.ks is not None else dout
            g = (g * ctx.scale).reshape(-1, table.shape[1])
            table.grad.index_add_(0, tok.reshape(-1), g.to(table.grad.dtype))
        _ready(rt, table)
        return None, None, None, None, None, None


# =============================================================================== attention (CPU reference core)
def _ref_attn_fwd(q, k, v, kv_len, causal, scale):
    """q [B,Lq,H,hd] ... -> out [B,Lq,H,hd], probs [B,H,Lq,Lk]. Masked logits
    get -1e9 added exactly as the reference does (transformer_model.py:101-102)."""
    s = torch.einsum("bqhd,bkhd->bhqk", q, k) * scale
    B, H, Lq, Lk = s.shape
    mask = torch.zeros(B, 1, Lq, Lk, dtype=s.dtype, device=s.device)
    keys = torch.arange(Lk, device=s.device)
    if kv_len is not None:
        mask = mask + (keys.view(1, 1, 1, Lk) >= kv_len.view(B, 1, 1, 1).to(keys.device)).to(s.dtype)
    if causal:
        qs = torch.arange(Lq, device=s.device)
        mask = torch.maximum(mask, (keys.view(1, Lk) > qs.view(Lq, 1)).to(s.dtype).view(1, 1, Lq, Lk))
    p = torch.softmax(s + mask * -1e9, dim=-1)
    out = torch.einsum("bhqk,bkhd->bqhd", p, v)
    return out, p


def _ref_attn_bwd(q, k, v, p, dout, scale):
    dv = torch.einsum("bhqk,bqhd->bkhd", p, dout)
    dp = torch.einsum("bqhd,bkhd->bhqk", dout, v)
    ds = p * (dp - (dp * p).sum(-1, keepdim=True))
    dq = torch.einsum("bhqk,bkhd->bqhd", ds, k) * scale
    dk = torch.einsum("bhqk,bqhd->bkhd", ds, q) * scale
    return dq, dk, dv


def attention_probs(q, k, kv_len, causal: bool, scale: float) -> torch.Tensor:
    """Attention weights [B,H,Lq,Lk] (f32), the maps the reference returns."""
    if q.is_cuda:
        return K.attn_probs(q, k, kv_len, scale, causal)
    return _ref_attn_fwd(q, k, k, kv_len, causal, scale)[1]


# =============================================================================== self-attention block
class SelfAttnBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wqkv: Param, bqkv: Param, wo: Param, bo: Param, gamma: Param,
                beta: Param, heads: int, kv_len, causal: bool, site: int, rt: RunCtx):
        B, L, d = x.shape
        hd = d // heads
        scale = 1.0 / math.sqrt(hd)
        ctx.p = (wqkv, bqkv, wo, bo, gamma, beta)
        ctx.meta = (heads, causal, scale, site, rt)
        x2 = x.reshape(B * L, d)
        ctx.lean = lean = x.is_cuda and _attn_lean(rt, B * L, wqkv, wo, d)
        kx = [] if lean else None
        if x.is_cuda:
            f8 = rt.fp8 is not None and K.attn_fwd_fp8_ok(L, L, hd)
            # the fp8 backward reads only the e4m3 Q|K|V: no bf16 copy then
            ctx.f8b = f8 and _f8_bwd_planned(rt, lean, L, L, hd)
            r = (rt.fp8.linear(x2, wqkv, bqkv, want8=f8, keep_x8=kx, want_y=not ctx.f8b)
                 if rt.fp8 is not None else None)
            qkv, qkv8 = (r[0], r[1]) if f8 and r is not None else (r, None)
            fused = None
            if qkv is None and not ctx.f8b and rt.fp8 is None and rt.attn_maps is None:
                # projection + attention forward in one launch (L <= 128)
                fused = K.qkv_attn_fwd(x2, wqkv.compute, bqkv.master, B, heads, kv_len, scale, causal)
                if fused is not None:
                    qkv = fused[0]
            if qkv is None and not ctx.f8b:
                qkv = K.linear_fwd(x2, wqkv.compute, bqkv.master)  # [M, 3d]
            q5 = qkv.view(B, L, 3, heads, hd) if qkv is not None else None
            o8e = None
            ctx.q8 = None
            if fused is not None:
                o, aux = fused[1], fused[2]
            elif qkv8 is not None:  # e4m3 attention on the projection's e4m3 output
                q85 = qkv8.view(B, L, 3, heads, hd)
                s8 = rt.fp8.meta.s(r[2])
                ctx.q8 = (qkv8, r[2])  # (the fp8 attention backward's operands)
                # (lean: the epilogue also emits the e4m3 O of the output projection)
                o8e = rt.fp8.o8_for(wo, (B, L, heads, hd), x.device) if lean else None
                o, aux = K.attn_fwd_fp8(q85[:, :, 0], q85[:, :, 1], q85[:, :, 2], s8, s8, s8, kv_len,
                                        scale, causal, *(o8e or ()))
            else:
                o, aux = K.attn_fwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], kv_len, scale, causal)
            s = None  # projection fused with the LayerNorm below
        else:
            qkv = x2 @ wqkv.master.t() + bqkv.master
            q5 = qkv.view(B, L, 3, heads, hd)
            o, aux = _ref_attn_fwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], kv_len, causal, scale)
            s = o.reshape(B * L, d) @ wo.master.t() + bo.master
        if rt.attn_maps is not None:  # (_f8_bwd_planned: q5 exists when maps are asked for)
            rt.attn_maps[site] = attention_probs(q5[:, :, 0], q5[:, :, 1], kv_len, causal, scale)
        ctx.f8a = None
        if lean:  # e4m3 output projection; keep the e4m3 operands for the backward
            s, o8 = rt.fp8.out_proj(o.view(B * L, d), wo, bo, o8e[0] if o8e else None)
            ctx.f8a = (kx[0], kx[1], o8)
            y, ctx.ln = _ln_fwd(x, s.view(B, L, d), gamma, beta, site, rt)
        elif s is None:
            y, ctx.ln = _proj_ln_fwd(o.view(B * L, d), wo, bo, x, gamma, beta, site, rt)
        else:
            y, ctx.ln = _ln_fwd(x, s.view(B, L, d), gamma, beta, site, rt)
        ctx.save_for_backward(x2, qkv, o, aux, kv_len)
        return y

    @staticmethod
    def backward(ctx, dy):
        wqkv, bqkv, wo, bo, gamma, beta = ctx.p
        heads, causal, scale, site, rt = ctx.meta
        x2, qkv, o, aux, kv_len = ctx.saved_tensors
        B, L, d = dy.shape
        M = B * L
        hd = d // heads
        bt = _beta(rt)
        if ctx.lean:
            return SelfAttnBlockFn._backward_fp8(ctx, dy)
        dh, ds = _ln_bwd(dy, ctx.ln, gamma, beta, bo, site, rt)
        ds2 = ds.reshape(M, d)
        q5 = qkv.view(B, L, 3, heads, hd)
        if dy.is_cuda:
            _wgrad(rt, ds2, o.view(M, d), d, wo)
            dqkv = torch.empty(M, 3 * d, dtype=torch.bfloat16, device=dy.device)
            g5 = dqkv.view(B, L, 3, heads, hd)
            # (L <= 128: the output projection's dgrad dO = ds @ Wo inside the
            # attention backward)
            if not K.attn_bwd_fdo(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o, ds2, wo.compute, aux,
                                  g5[:, :, 0], g5[:, :, 1], g5[:, :, 2], kv_len, scale, causal):
                do = K.linear_dgrad(ds2, wo.compute, d)
                K.attn_bwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o, do.view(B, L, heads, hd), aux,
                           g5[:, :, 0], g5[:, :, 1], g5[:, :, 2], kv_len, scale, causal)
            _wgrad(rt, dqkv, x2, 3 * d, wqkv, bqkv)
            dx = _dgrad_res(dqkv, wqkv, 3 * d, dh)
            if rt.wgrad is not None:
                rt.wgrad.layer_end()  # self-attention is a layer's first block
            return (dx.view(B, L, d),) + (None,) * 11
        else:
            _write_grad(wo, ds2.t() @ o.reshape(M, d), rt)
            _ready(rt, wo)
            do = (ds2 @ wo.master).view(B, L, heads, hd)
            dq, dk, dv = _ref_attn_bwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], aux, do, scale)
            dqkv = torch.stack([dq, dk, dv], dim=2).reshape(M, 3 * d)
            _write_grad(wqkv, dqkv.t() @ x2, rt)
            _write_grad(bqkv, dqkv.sum(0), rt)
        _ready(rt, wqkv, bqkv)
        dx = _dgrad_into(dqkv, wqkv, 3 * d, dh)
        return (dx.view(B, L, d),) + (None,) * 11

    @staticmethod
    def _backward_fp8(ctx, dy):
        """Lean fp8 backward: e5m2 ds from the LayerNorm backward -> O-proj
        dgrad (e5m2 x e4m3 Wo^T) -> bf16 attention backward -> e5m2 dQ|dK|dV
        -> input-projection dgrad (into the residual gradient); both weight
        gradients in fp8 from the saved e4m3 operands."""
        wqkv, bqkv, wo, bo, gamma, beta = ctx.p
        heads, causal, scale, site, rt = ctx.meta
        x2, qkv, o, aux, kv_len = ctx.saved_tensors
        B, L, d = dy.shape
        M, hd, bt = B * L, d // heads, _beta(rt)
        st = rt.fp8
        x8, xs, o8 = ctx.f8a
        os_, go = st.attn_out[id(wo)]
        dh, ds8 = _ln_bwd(dy, ctx.ln, gamma, beta, bo, site, rt, ds8_slot=go)
        ds8 = ds8.view(M, d)
        gq = st.proj_bwd[id(wqkv)]
        if _attn_f8_bwd(ctx, L, L, hd):
            # fp8 attention backward: e5m2 dO straight from the output
            # projection's dgrad, e4m3 Q/K/V of the forward -> e5m2 dQ|dK|dV
            gdo, gds = st.attn_bwd8[id(wo)]
            do8 = _fp8_dgrad8(ds8, go, wo, gdo, rt)
            qkv8, qs = ctx.q8
            q85 = qkv8.view(B, L, 3, heads, hd)
            s8 = st.meta.s(qs)
            dqkv8 = torch.empty(M, 3 * d, dtype=st.gmeta.dtype, device=dy.device)
            g85 = dqkv8.view(B, L, 3, heads, hd)
            part = K.workspace(f"f8cs_qkv{site}", B * 3 * d, dy.device)
            nparts = K.attn_bwd_f8(q85[:, :, 0], q85[:, :, 1], q85[:, :, 2], s8, s8, s8, o,
                                   do8.view(B, L, heads, hd), st.gmeta.s(gdo), aux, kv_len, scale,
                                   causal, st.gmeta.s(gds), st.gmeta.a(gds), dq8=g85[:, :, 0],
                                   dk8=g85[:, :, 1], dv8=g85[:, :, 2], sg8=st.gmeta.s(gq),
                                   amaxg8=st.gmeta.a(gq), cs_part=part, cs_ld=3 * d, cs_q=0,
                                   cs_k=d, cs_v=2 * d)
            _fold_bias_later(rt, part[: nparts * 3 * d], nparts, 3 * d, bqkv)
            return SelfAttnBlockFn._finish_fp8(ctx, rt, st, dh, ds8, go, dqkv8, gq, x8, xs, o8, os_,
                                               M, d, B, L, bt)
        do = torch.empty(M, d, dtype=torch.bfloat16, device=dy.device)
        _fp8_dgrad_into(ds8, go, wo, do, rt, 0.0)
        q5 = qkv.view(B, L, 3, heads, hd)
        dqkv = torch.empty(M, 3 * d, dtype=torch.bfloat16, device=dy.device)
        g5 = dqkv.view(B, L, 3, heads, hd)
        if fp8.ATTN_BWD_G8 and K.attn_bwd_g8_ok(L, L, hd):
            # the attention backward emits e5m2 dQ|dK|dV, their amax and the
            # bias-gradient partials itself (no bf16 dQ|dK|dV pass)
            dqkv8 = torch.empty(M, 3 * d, dtype=st.gmeta.dtype, device=dy.device)
            g85 = dqkv8.view(B, L, 3, heads, hd)
            part = K.workspace(f"qcs_qkv{site}", B * -(-L // 128) * 3 * d, dy.device)
            nparts = K.attn_bwd_g8(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o, do.view(B, L, heads, hd),
                                   aux, g5[:, :, 0], g5[:, :, 1], g5[:, :, 2], kv_len, scale, causal,
                                   g85[:, :, 0], g85[:, :, 1], g85[:, :, 2], st.gmeta.s(gq),
                                   st.gmeta.a(gq), part, 3 * d, 0, d, 2 * d)
            _fold_bias_later(rt, part[: nparts * 3 * d], nparts, 3 * d, bqkv)
        else:
            K.attn_bwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o, do.view(B, L, heads, hd), aux,
                       g5[:, :, 0], g5[:, :, 1], g5[:, :, 2], kv_len, scale, causal)
            dqkv8 = _fp8_grad_bias(dqkv, gq, bqkv, rt, f"qkv{site}")
        return SelfAttnBlockFn._finish_fp8(ctx, rt, st, dh, ds8, go, dqkv8, gq, x8, xs, o8, os_, M,
                                           d, B, L, bt)

    @staticmethod
    def _finish_fp8(ctx, rt, st, dh, ds8, go, dqkv8, gq, x8, xs, o8, os_, M, d, B, L, bt):
        """input-projection dgrad into the residual gradient, both weight
        gradients in fp8"""
        wqkv, bqkv, wo = ctx.p[0], ctx.p[1], ctx.p[2]
        _fp8_dgrad_into(dqkv8, gq, wqkv, dh.view(M, d), rt, 1.0)
        q = rt.wgrad
        q.add_fp8(ds8, st.gmeta.s(go), o8, st.meta.s(os_), wo, bt, rt)
        q.add_fp8(dqkv8, st.gmeta.s(gq), x8, st.meta.s(xs), wqkv, bt, rt)
        q.layer_end()  # self-attention is a layer's first block
        return (dh.view(B, L, d),) + (None,) * 11


# =============================================================================== cross-attention
def _take_dkv(dkv_in, kvh: KVGrad, rows: int) -> torch.Tensor:
    """The batched d(K|V) [rows, layers * 2d] the decoder layers filled (layer
    0 also hands it to autograd, which delivers it as dkv_in)."""
    dkv = (dkv_in if dkv_in is not None else kvh.buf).reshape(rows, -1)
    kvh.buf = None
    return dkv


class CrossKVFn(torch.autograd.Function):
    """kv_all[B, S, layers*2*d] = enc @ Wkv_all^T + b: the K and V projections
    of the encoder output for every decoder layer in one GEMM."""

    @staticmethod
    def forward(ctx, enc, wkv: Param, bkv: Param, kvh: KVGrad, rt: RunCtx):
        B, S, d = enc.shape
        e2 = enc.reshape(B * S, d)
        ctx.p = (wkv, bkv)
        ctx.kvh, ctx.rt, ctx.shape = kvh, rt, (B, S, d)
        ctx.save_for_backward(e2)
        ctx.lean = lean = enc.is_cuda and _attn_lean(rt, B * S, wkv, None, d)
        kx = [] if lean else None
        ctx.f8a = None
        T = kvh.dec_len
        hd = d // kvh.heads if kvh.heads else 0
        # every decoder layer's cross-attention runs e4m3 forward + fp8
        # backward: the bf16 K|V are never read (and d(K|V) come as e5m2)
        kvh.f8b = bool(lean and enc.is_cuda and T and K.attn_fwd_fp8_ok(T, S, hd)
                       and fp8.wgrad_fp8_ok(B * T, d, d) and _f8_bwd_planned(rt, True, T, S, hd))
        if enc.is_cuda:
            kv = None
            if rt.fp8 is not None:
                r = rt.fp8.linear(e2.contiguous(), wkv, bkv, want8=True, keep_x8=kx, want_y=not kvh.f8b)
                if lean and r is not None:
                    ctx.f8a = tuple(kx)
                if r is not None:  # its e4m3 copy feeds the decoders' e4m3 attention
                    kv = r[0]
                    rt.fp8.kv8 = (r[1].view(B, S, -1), r[2])
                    if kvh.f8b:  # (autograd needs an output of this shape; nothing reads
                        # it: a zero-stride placeholder, not a bf16 K|V image)
                        kv = torch.zeros(1, dtype=torch.bfloat16, device=enc.device).expand(
                            B * S, r[1].shape[1])
            if kv is None:
                kv = K.linear_fwd(e2.contiguous(), wkv.compute, bkv.master)
        else:
            kv = e2 @ wkv.master.t() + bkv.master
        return kv.view(B, S, -1)

    @staticmethod
    def backward(ctx, dkv_in):
        wkv, bkv = ctx.p
        rt = ctx.rt
        B, S, d = ctx.shape
        (e2,) = ctx.saved_tensors
        # filled slice-by-slice by every CrossAttnBlockFn.backward (layer 0
        # also hands it to autograd, which delivers it here as dkv_in)
        kvh = ctx.kvh
        N = wkv.shape[0]
        bt = _beta(rt)
        if e2.is_cuda and ctx.f8a is not None:
            # lean fp8: e5m2 dK|dV of every decoder layer -> one dgrad + fp8
            # weight gradient against the encoder output's e4m3 copy
            st = rt.fp8
            x8, xs = ctx.f8a
            gk = st.proj_bwd[id(wkv)]
            if kvh.f8b:  # written by the layers' fp8 attention backward (e5m2 + bias sums;
                # dkv_in is the layers' zero-stride placeholder)
                dkv8 = kvh.buf8.reshape(B * S, -1)
                _fold_bias_later(rt, kvh.part, B, N, bkv)
                kvh.buf8 = kvh.part = None
            else:
                dkv8 = _fp8_grad_bias(_take_dkv(dkv_in, kvh, B * S).contiguous(), gk, bkv, rt, "kv")
            rt.wgrad.add_fp8(dkv8, st.gmeta.s(gk), x8, st.meta.s(xs), wkv, bt, rt)
            rt.wgrad.boundary()
            denc = torch.empty(B * S, d, dtype=torch.bfloat16, device=e2.device)
            _fp8_dgrad_into(dkv8, gk, wkv, denc, rt, 0.0)
            if rt.store is not None:
                rt.store.release_point()
            return denc.view(B, S, d), None, None, None, None
        dkv = _take_dkv(dkv_in, kvh, B * S)
        if e2.is_cuda:
            _wgrad(rt, dkv, e2, N, wkv, bkv)
            if rt.wgrad is not None:
                rt.wgrad.boundary()  # every decoder layer's backward is done
            denc = _dgrad_res(dkv, wkv, N, None)
        else:
            _write_grad(wkv, dkv.t() @ e2, rt)
            _write_grad(bkv, dkv.sum(0), rt)
            _ready(rt, wkv, bkv)
            denc = dkv @ wkv.master
        if rt.store is not None:
            # the rest of backward (encoder) reads no decoder-side weight: the
            # data-parallel optimizer may update those buckets from here on
            rt.store.release_point()
        return denc.view(B, S, d), None, None, None, None


class CrossAttnBlockFn(torch.autograd.Function):
    """Decoder block 2: Q from the decoder stream, K = V = encoder output
    (reference call order mha2(enc, enc, out1) -> values, keys, query)."""

    @staticmethod
    def forward(ctx, x, kv_all, layer: int, kvh: KVGrad, wq: Param, bq: Param, wo: Param,
                bo: Param, gamma: Param, beta: Param, heads: int, kv_len, site: int, rt: RunCtx):
        B, T, d = x.shape
        S = kv_all.shape[1]
        hd = d // heads
        scale = 1.0 / math.sqrt(hd)
        ctx.p = (wq, bq, wo, bo, gamma, beta)
        ctx.meta = (heads, scale, site, rt, layer, kvh)
        x2 = x.reshape(B * T, d)
        kv5 = None  # (kvh.f8b: kv_all is a placeholder, the e4m3 K|V are read)
        if not kvh.f8b:
            if not kv_all.is_contiguous():
                raise ValueError("kv_all must be contiguous")
            kv5 = kv_all[:, :, layer * 2 * d:(layer + 1) * 2 * d].view(B, S, 2, heads, hd)
        ctx.lean = lean = x.is_cuda and _attn_lean(rt, B * T, wq, wo, d)
        kx = [] if lean else None
        if x.is_cuda:
            o8e = None
            f8 = (rt.fp8 is not None and rt.fp8.kv8 is not None and K.attn_fwd_fp8_ok(T, S, hd))
            ctx.f8b = f8 and _f8_bwd_planned(rt, lean, T, S, hd)
            if kvh.f8b and not ctx.f8b:
                raise RuntimeError("cross-attention: the batched K|V were produced for the fp8 "
                                   "backward (no bf16 copy) but this layer does not run it")
            r = (rt.fp8.linear(x2, wq, bq, want8=f8, keep_x8=kx, want_y=not ctx.f8b)
                 if rt.fp8 is not None else None)
            q, q8 = (r[0], r[1]) if f8 and r is not None else (r, None)
            fused = None
            if q is None and not ctx.f8b and rt.fp8 is None and rt.attn_maps is None and kv5 is not None:
                # Q projection + attention forward in one launch (<= 128 tokens)
                fused = K.qkv_attn_fwd(x2, wq.compute, bq.master, B, heads, kv_len, scale, False,
                                       k=kv5[:, :, 0], v=kv5[:, :, 1])
                if fused is not None:
                    q = fused[0]
            if q is None and not ctx.f8b:
                q = K.linear_fwd(x2, wq.compute, bq.master)
            ctx.q8 = None
            if fused is not None:
                o, aux = fused[1], fused[2]
            elif q8 is not None:  # e4m3 attention: e4m3 Q and the batched e4m3 K|V
                kv8, kvs = rt.fp8.kv8
                if kv8.shape != kv_all.shape:
                    raise RuntimeError(f"fp8 cross K|V {tuple(kv8.shape)} is not this forward's "
                                       f"{tuple(kv_all.shape)}")
                kv85 = kv8[:, :, layer * 2 * d:(layer + 1) * 2 * d].view(B, S, 2, heads, hd)
                skv = rt.fp8.meta.s(kvs)
                ctx.q8 = (q8, r[2], kv85, kvs)  # (the fp8 attention backward's operands)
                o8e = rt.fp8.o8_for(wo, (B, T, heads, hd), x.device) if lean else None
                o, aux = K.attn_fwd_fp8(q8.view(B, T, heads, hd), kv85[:, :, 0], kv85[:, :, 1],
                                        rt.fp8.meta.s(r[2]), skv, skv, kv_len, scale, False,
                                        *(o8e or ()))
            else:
                o, aux = K.attn_fwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], kv_len,
                                    scale, False)
            s = None  # projection fused with the LayerNorm below
        else:
            q = x2 @ wq.master.t() + bq.master
            o, aux = _ref_attn_fwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], kv_len,
                                   False, scale)
            s = o.reshape(B * T, d) @ wo.master.t() + bo.master
        if rt.attn_maps is not None:  # (_f8_bwd_planned: q exists when maps are asked for)
            rt.attn_maps[site] = attention_probs(q.view(B, T, heads, hd), kv5[:, :, 0], kv_len, False, scale)
        ctx.f8a = None
        if lean:  # e4m3 output projection; keep the e4m3 operands for the backward
            s, o8 = rt.fp8.out_proj(o.view(B * T, d), wo, bo, o8e[0] if o8e else None)
            ctx.f8a = (kx[0], kx[1], o8)
            y, ctx.ln = _ln_fwd(x, s.view(B, T, d), gamma, beta, site, rt)
        elif s is None:
            y, ctx.ln = _proj_ln_fwd(o.view(B * T, d), wo, bo, x, gamma, beta, site, rt)
        else:
            y, ctx.ln = _ln_fwd(x, s.view(B, T, d), gamma, beta, site, rt)
        ctx.save_for_backward(x2, kv_all, q, o, aux, kv_len)
        return y

    @staticmethod
    def backward(ctx, dy):
        wq, bq, wo, bo, gamma, beta = ctx.p
        heads, scale, site, rt, layer, kvh = ctx.meta
        x2, kv_all, q, o, aux, kv_len = ctx.saved_tensors
        B, T, d = dy.shape
        S = kv_all.shape[1]
        hd = d // heads
        bt = _beta(rt)
        M = B * T
        if kvh.f8b:
            # every layer's d(K|V) goes to kvh.buf8 as e5m2: autograd gets a
            # zero-stride placeholder of the right shape, no bf16 buffer
            dkv_all = kv5 = g5 = None
        else:
            if kvh.buf is None:
                kvh.buf = torch.empty(B * S, kv_all.shape[2], dtype=kv_all.dtype, device=dy.device)
            dkv_all = kvh.buf.view(B, S, -1)
            kv5 = kv_all[:, :, layer * 2 * d:(layer + 1) * 2 * d].view(B, S, 2, heads, hd)
            g5 = dkv_all[:, :, layer * 2 * d:(layer + 1) * 2 * d].view(B, S, 2, heads, hd)
        if ctx.lean:
            st = rt.fp8
            x8, xs, o8 = ctx.f8a
            os_, go = st.attn_out[id(wo)]
            dh, ds8 = _ln_bwd(dy, ctx.ln, gamma, beta, bo, site, rt, ds8_slot=go)
            ds8 = ds8.view(M, d)
            gq = st.proj_bwd[id(wq)]
            if _attn_f8_bwd(ctx, T, S, hd):
                # fp8 attention backward: e5m2 dQ (+ amax, bias sums); dK / dV
                # as e5m2 into kvh.buf8 (kvh.f8b) or bf16 into the batched
                # cross K|V gradient
                gdo, gds = st.attn_bwd8[id(wo)]
                do8 = _fp8_dgrad8(ds8, go, wo, gdo, rt)
                q8, qs, kv85, kvs = ctx.q8
                skv = st.meta.s(kvs)
                dq8 = torch.empty(M, d, dtype=st.gmeta.dtype, device=dy.device)
                part = K.workspace(f"f8cs_q{site}", B * d, dy.device)
                if kvh.f8b:
                    # e5m2 d(K|V) straight into the batched buffer (the cross K|V
                    # projection's gradient slot), bias sums into kvh.part
                    NKV = kv_all.shape[2]
                    if kvh.buf8 is None:
                        kvh.buf8 = torch.empty(B, S, NKV, dtype=st.gmeta.dtype, device=dy.device)
                        kvh.part = torch.empty(B, NKV, dtype=torch.float32, device=dy.device)
                    g85 = kvh.buf8[:, :, layer * 2 * d:(layer + 1) * 2 * d].view(B, S, 2, heads, hd)
                    gk = st.proj_bwd[id(kvh.wkv)]
                    kvo = dict(dk8=g85[:, :, 0], dv8=g85[:, :, 1], sgkv8=st.gmeta.s(gk),
                               amaxgkv8=st.gmeta.a(gk), cs_part2=kvh.part, cs_ld2=NKV,
                               cs_k=layer * 2 * d, cs_v=layer * 2 * d + d)
                else:
                    kvo = dict(dk=g5[:, :, 0], dv=g5[:, :, 1])
                nparts = K.attn_bwd_f8(q8.view(B, T, heads, hd), kv85[:, :, 0], kv85[:, :, 1],
                                       st.meta.s(qs), skv, skv, o, do8.view(B, T, heads, hd),
                                       st.gmeta.s(gdo), aux, kv_len, scale, False, st.gmeta.s(gds),
                                       st.gmeta.a(gds), dq8=dq8.view(B, T, heads, hd),
                                       sg8=st.gmeta.s(gq), amaxg8=st.gmeta.a(gq), cs_part=part,
                                       cs_ld=d, cs_q=0, **kvo)
                _fold_bias_later(rt, part[: nparts * d], nparts, d, bq)
                _fp8_dgrad_into(dq8, gq, wq, dh.view(M, d), rt, 1.0)
                rt.wgrad.add_fp8(ds8, st.gmeta.s(go), o8, st.meta.s(os_), wo, bt, rt)
                rt.wgrad.add_fp8(dq8, st.gmeta.s(gq), x8, st.meta.s(xs), wq, bt, rt)
                dkv_ret = None
                if layer == 0:
                    dkv_ret = dkv_all if dkv_all is not None else torch.zeros(
                        1, dtype=kv_all.dtype, device=dy.device).expand(kv_all.shape)
                return (dh.view(B, T, d), dkv_ret) + (None,) * 12
            do = torch.empty(M, d, dtype=torch.bfloat16, device=dy.device)
            _fp8_dgrad_into(ds8, go, wo, do, rt, 0.0)
            dq = torch.empty(M, d, dtype=torch.bfloat16, device=dy.device)
            if fp8.ATTN_BWD_G8 and K.attn_bwd_g8_ok(T, S, hd):
                # e5m2 dQ (+ amax, bias partials) from the attention backward;
                # dK / dV stay bf16 (summed over the layers into the batched
                # cross K|V gradient)
                dq8 = torch.empty(M, d, dtype=st.gmeta.dtype, device=dy.device)
                part = K.workspace(f"qcs_q{site}", B * -(-T // 128) * d, dy.device)
                nparts = K.attn_bwd_g8(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], o,
                                       do.view(B, T, heads, hd), aux, dq.view(B, T, heads, hd),
                                       g5[:, :, 0], g5[:, :, 1], kv_len, scale, False,
                                       dq8.view(B, T, heads, hd), None, None, st.gmeta.s(gq),
                                       st.gmeta.a(gq), part, d, 0, 0, 0, skip_bf16=False)
                _fold_bias_later(rt, part[: nparts * d], nparts, d, bq)
            else:
                K.attn_bwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], o,
                           do.view(B, T, heads, hd), aux, dq.view(B, T, heads, hd), g5[:, :, 0],
                           g5[:, :, 1], kv_len, scale, False)
                dq8 = _fp8_grad_bias(dq, gq, bq, rt, f"q{site}")
            _fp8_dgrad_into(dq8, gq, wq, dh.view(M, d), rt, 1.0)
            rt.wgrad.add_fp8(ds8, st.gmeta.s(go), o8, st.meta.s(os_), wo, bt, rt)
            rt.wgrad.add_fp8(dq8, st.gmeta.s(gq), x8, st.meta.s(xs), wq, bt, rt)
            dkv_ret = dkv_all if layer == 0 else None
            return (dh.view(B, T, d), dkv_ret) + (None,) * 12
        dh, ds = _ln_bwd(dy, ctx.ln, gamma, beta, bo, site, rt)
        ds2 = ds.reshape(M, d)
        if dy.is_cuda:
            _wgrad(rt, ds2, o.view(M, d), d, wo)
            dq = torch.empty(M, d, dtype=torch.bfloat16, device=dy.device)
            if not K.attn_bwd_fdo(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], o, ds2,
                                  wo.compute, aux, dq.view(B, T, heads, hd), g5[:, :, 0],
                                  g5[:, :, 1], kv_len, scale, False):
                do = K.linear_dgrad(ds2, wo.compute, d)
                K.attn_bwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], o,
                           do.view(B, T, heads, hd), aux, dq.view(B, T, heads, hd), g5[:, :, 0],
                           g5[:, :, 1], kv_len, scale, False)
            _wgrad(rt, dq, x2, d, wq, bq)
        else:
            _write_grad(wo, ds2.t() @ o.reshape(M, d), rt)
            _ready(rt, wo)
            do = (ds2 @ wo.master).view(B, T, heads, hd)
            dqh, dk, dv = _ref_attn_bwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], aux,
                                        do, scale)
            g5[:, :, 0] = dk
            g5[:, :, 1] = dv
            dq = dqh.reshape(M, d)
            _write_grad(wq, dq.t() @ x2, rt)
            _write_grad(bq, dq.sum(0), rt)
            _ready(rt, wq, bq)  # (GPU: reported by _wgrad / the deferred flush)
        dx = _dgrad_res(dq, wq, d, dh)
        # Only layer 0 hands the (by then complete) shared buffer to autograd;
        # the other layers contribute through the side channel, so no adds.
        dkv_ret = dkv_all if layer == 0 else None
        return (dx.view(B, T, d), dkv_ret) + (None,) * 12


# =============================================================================== feed-forward block
class FFNBlockFn(torch.autograd.Function):
    """y = LN(x + dropout(Dense(d)(Dense(ff, relu)(x))))."""

    @staticmethod
    def forward(ctx, x, w1: Param, b1: Param, w2: Param, b2: Param, gamma: Param, beta: Param,
                site: int, rt: RunCtx):
        B, L, d = x.shape
        x2 = x.reshape(B * L, d)
        ctx.p = (w1, b1, w2, b2, gamma, beta)
        ctx.meta = (site, rt)
        ctx.f8 = None
        ctx.lean = False
        if x.is_cuda and rt.fp8 is not None:
            st = rt.fp8
            xs, hs = st.ffn_slots[id(w1)]
            w1_8, s1 = st.weights.get(w1)
            w2_8, s2 = st.weights.get(w2)
            x8 = st.stash.pop(xs, None)  # fused into the producing LayerNorm
            if x8 is None:
                x8 = fp8.quantize(x2, st.meta, xs)
            x8 = x8.view(x2.shape)
            # lean: the backward runs entirely on the e4m3 copies (fp8 weight
            # gradients, ReLU mask from h8), so the bf16 hidden is not written
            lean = (rt.training and rt.wgrad is not None and fp8.WGRAD_FP8
                    and st.ffn_bwd_slots.get(id(w1)) is not None
                    and fp8.wgrad_fp8_ok(B * L, d, w1.shape[0]))
            h, h8 = fp8.gemm_fp8(x8, w1_8, b1.master, st.meta, xs, s1, relu=True, out8_slot=hs,
                                 want_y=not lean)
            f, _ = fp8.gemm_fp8(h8, w2_8, b2.master, st.meta, hs, s2)
            # the e4m3 copies feed the fp8 weight gradients of the backward
            ctx.f8 = (x8, h8) if rt.training else None
            ctx.lean = lean
        elif x.is_cuda:
            h = K.linear_fwd(x2, w1.compute, b1.master, relu=True)
            f = None  # second projection fused with the LayerNorm below
        else:
            h = torch.relu(x2 @ w1.master.t() + b1.master)
            f = h @ w2.master.t() + b2.master
        if f is None:
            y, ctx.ln = _proj_ln_fwd(h, w2, b2, x, gamma, beta, site, rt)
        else:
            y, ctx.ln = _ln_fwd(x, f.view(B, L, d), gamma, beta, site, rt)
        ctx.save_for_backward(x2, h if h is not None else x2)  # (lean: h unused)
        return y

    @staticmethod
    def backward(ctx, dy):
        w1, b1, w2, b2, gamma, beta = ctx.p
        site, rt = ctx.meta
        x2, h = ctx.saved_tensors
        B, L, d = dy.shape
        ff = w1.shape[0]
        bt = _beta(rt)
        f8w = ctx.lean
        bw = rt.fp8.ffn_bwd_slots.get(id(w1)) if (dy.is_cuda and rt.fp8 is not None) else None
        # lean fp8 backward: the LayerNorm backward emits ds directly in e5m2
        dh, ds = _ln_bwd(dy, ctx.ln, gamma, beta, b2, site, rt, ds8_slot=bw[0] if f8w else None)
        ds2 = ds.reshape(B * L, d)
        if dy.is_cuda:
            if not f8w:
                _wgrad(rt, ds2, h, d, w2)
            if bw is not None:
                # fp8 backward: e5m2 gradients x e4m3 weights on the
                # block-scaled MFMA; the ReLU-backward dgrad also emits the e5m2
                # copy of its output for the next dgrad, which accumulates the
                # residual gradient already in dh
                st = rt.fp8
                gs, gh = bw
                M = B * L
                ds8 = ds2 if f8w else fp8.quantize(ds2, st.gmeta, gs)
                wp = fp8.DGRAD_PLAIN_W  # plain e4m3 weights read N-contiguous
                w2t8, s2t = st.weights.get(w2, transposed=not wp)
                w1t8, s1t = st.weights.get(w1, transposed=not wp)
                if f8w:
                    # lean fp8 backward: the ReLU-backward dgrad writes only
                    # the e5m2 dpre8 and, from its epilogue, b1's gradient
                    # (column sums); the mask is the forward's e4m3 hidden h8;
                    # weight gradients: e5m2 gradients x the forward's e4m3
                    # inputs (FFN1 input x8, hidden h8), token-major
                    x8, h8 = ctx.f8
                    xs, hs = st.ffn_slots[id(w1)]
                    q = rt.wgrad
                    # (b1's column-sum fold deferred to the wgrad flush with
                    # the LayerNorm folds: one launch instead of one per layer)
                    dpre8 = fp8.gemm_bf8_dgrad(ds8, st.gmeta, gs, w2t8, st.meta, s2t, None,
                                               relu_aux8=h8.view(M, ff), out8_slot=gh,
                                               colsum_out=b1.grad, colsum_beta=bt, w_plain=wp,
                                               defer=q.reductions)
                    q.reduced_params.append((rt, b1))
                    q.add_fp8(ds8.view(M, d), st.gmeta.s(gs), h8.view(M, ff), st.meta.s(hs), w2, bt, rt)
                    q.add_fp8(dpre8.view(M, ff), st.gmeta.s(gh), x8.view(M, d), st.meta.s(xs), w1, bt, rt)
                else:
                    dpre = torch.empty(M, ff, dtype=ds2.dtype, device=ds2.device)
                    dpre8 = fp8.gemm_bf8_dgrad(ds8, st.gmeta, gs, w2t8, st.meta, s2t, dpre, relu_aux=h,
                                               out8_slot=gh, w_plain=wp)
                    _wgrad(rt, dpre, x2, ff, w1, b1)
                fp8.gemm_bf8_dgrad(dpre8, st.gmeta, gh, w1t8, st.meta, s1t, dh.view(M, d), beta=1.0,
                                   w_plain=wp)
                return (dh.view(B, L, d),) + (None,) * 8
            if w2.compute_t is not None and not w2.compute_t_stale:
                # NT layout against W2^T (ParamStore.add_transposed; stale while
                # an fp8 backward had the re-transposes paused: NN below)
                dpre = K.linear_dgrad_t(ds2, w2.compute_t, relu_aux=h)
            else:
                dpre = K.linear_dgrad(ds2, w2.compute, d, relu_aux=h)
            _wgrad(rt, dpre, x2, ff, w1, b1)
            dx = _dgrad_res(dpre, w1, ff, dh)
            return (dx.view(B, L, d),) + (None,) * 8
        else:
            _write_grad(w2, ds2.t() @ h, rt)
            _ready(rt, w2)
            dpre = (ds2 @ w2.master) * (h > 0).to(ds2.dtype)
            _write_grad(w1, dpre.t() @ x2, rt)
            _write_grad(b1, dpre.sum(0), rt)
        _ready(rt, w1, b1)
        dx = _dgrad_into(dpre, w1, ff, dh)
        return (dx.view(B, L, d),) + (None,) * 8
