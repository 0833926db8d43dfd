"""Fused layer-level autograd ops of the encoder-decoder Transformer.

Each op is a coarse `torch.autograd.Function` with a hand-written backward that
sequences the gfx950 kernels (GEMM with fused epilogues, flash attention,
fused dropout+residual+LayerNorm, fused embedding) and writes parameter
gradients straight into the flat f32 gradient buffer, notifying the
data-parallel engine as each one becomes final (so its bucket's all-reduce can
start while backward continues).

On CPU tensors the same ops run a plain-PyTorch f32 reference with identical
semantics (including the Philox dropout masks): that is the CPU test path and
the BASELINE "tiny on CPU" configuration; on GPU tensors only the HIP kernels
run.

Semantics follow the reference model
(reference: distributed_training_transformer/transformer_model.py):
  MultiHeadAttention :112-166  (separate Q/K/V Dense; here fused [3d,d] / [2d,d])
  FFN                :169-175  (Dense(ff, relu) -> Dense(d))
  post-LN sublayer   :187-204, :219-248  (LN(x + dropout(sublayer(x))), eps 1e-6)
  embedding          :270-279, :301-308  (emb * sqrt(d) + PE, dropout)
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

from tensorflow_distributed_on_gke_amd.models.params import Param, ParamStore
from tensorflow_distributed_on_gke_amd.ops import kernels as K
from tensorflow_distributed_on_gke_amd.ops import philox


@dataclass
class RunCtx:
    """Per-forward runtime state shared by all layers."""

    training: bool = False
    dropout: float = 0.1
    seed: int = 0
    ctr: Optional[torch.Tensor] = None  # int64[1]: dropout stream counter (device-resident)
    accumulate: bool = False  # accumulate into existing grads (gradient accumulation)
    store: Optional[ParamStore] = None

    @property
    def p(self) -> float:
        return self.dropout if self.training else 0.0

    def cpu_offset(self, site: int) -> int:
        c = int(self.ctr.item()) if self.ctr is not None else 0
        return philox.rng_offset(c, site) if self.ctr is not None else site


def _keep_scale(rt: RunCtx, site: int, shape, device) -> Optional[torch.Tensor]:
    """CPU reference dropout multiplier (keep/(1-p)) with the device RNG stream."""
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


# =============================================================================== embedding
class EmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, anchor, tok, table: Param, pe: torch.Tensor, site: int, rt: RunCtx):
        d = table.shape[1]
        scale = math.sqrt(d)
        ctx.table, ctx.site, ctx.rt, ctx.scale = table, site, rt, scale
        ctx.save_for_backward(tok)
        if tok.is_cuda:
            return K.embed_fwd(tok, table.compute, pe, scale, rt.p, rt.seed, rt.ctr, site)
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
            K.embed_bwd(tok, dout.contiguous(), table.grad, ctx.scale, rt.p, rt.seed, rt.ctr,
                        ctx.site)
        else:
            g = dout * ctx.ks if ctx.ks is not None else dout
            g = (g * ctx.scale).reshape(-1, table.shape[1])
            table.grad.index_add_(0, tok.reshape(-1), g.to(table.grad.dtype))
        _ready(rt, table)
        return None, None, None, None, None, None


# =============================================================================== residual + LN
class AddLNFn(torch.autograd.Function):
    """y = LayerNorm(x + dropout(s)); optionally also produces the bias grad of
    the sublayer that produced `s` (sum of ds over rows)."""

    @staticmethod
    def forward(ctx, x, s, gamma: Param, beta: Param, site: int, rt: RunCtx,
                sub_bias: Optional[Param]):
        ctx.gamma, ctx.beta, ctx.site, ctx.rt, ctx.sub_bias = gamma, beta, site, rt, sub_bias
        p = rt.p
        if x.is_cuda:
            y, h, mean, rstd = K.ln_fwd(x.contiguous(), s.contiguous(), gamma.master, beta.master,
                                        p, rt.seed, rt.ctr, site)
            ctx.save_for_backward(h, mean, rstd)
            return y
        ks = _keep_scale(rt, site, s.shape, s.device)
        h = x + (s * ks if ks is not None else s)
        mean = h.mean(-1, keepdim=True)
        var = ((h - mean) ** 2).mean(-1, keepdim=True)
        rstd = torch.rsqrt(var + 1e-6)
        ctx.ks = ks
        ctx.save_for_backward(h, mean, rstd)
        return (h - mean) * rstd * gamma.master + beta.master

    @staticmethod
    def backward(ctx, dy):
        h, mean, rstd = ctx.saved_tensors
        gamma, beta, rt, sb = ctx.gamma, ctx.beta, ctx.rt, ctx.sub_bias
        if dy.is_cuda:
            dh, ds = K.ln_bwd(dy.contiguous(), h, mean, rstd, gamma.master, gamma.grad, beta.grad,
                              sb.grad if sb is not None else None, rt.p, rt.seed, rt.ctr, ctx.site,
                              want_ds=True, accumulate=rt.accumulate)
        else:
            xhat = (h - mean) * rstd
            D = h.shape[-1]
            g = dy * gamma.master
            dh = rstd * (g - g.mean(-1, keepdim=True) - xhat * (g * xhat).mean(-1, keepdim=True))
            ds = dh * ctx.ks if ctx.ks is not None else dh
            _write_grad(gamma, (dy * xhat).reshape(-1, D).sum(0), rt)
            _write_grad(beta, dy.reshape(-1, D).sum(0), rt)
            if sb is not None:
                _write_grad(sb, ds.reshape(-1, D).sum(0), rt)
        _ready(rt, gamma, beta, *([sb] if sb is not None else []))
        return dh, ds, None, None, None, None, None


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


# =============================================================================== multi-head attention
class SelfMHAFn(torch.autograd.Function):
    """out = Dense_o(SDPA(Dense_q x, Dense_k x, Dense_v x)) with fused QKV."""

    @staticmethod
    def forward(ctx, x, wqkv: Param, bqkv: Param, wo: Param, bo: Param, heads: int,
                kv_len, causal: bool, rt: RunCtx, fused_bo_grad: bool):
        B, L, d = x.shape
        hd = d // heads
        scale = 1.0 / math.sqrt(hd)
        ctx.p = (wqkv, bqkv, wo, bo)
        ctx.meta = (heads, causal, scale, rt, fused_bo_grad)
        x2 = x.reshape(B * L, d)
        if x.is_cuda:
            qkv = K.linear_fwd(x2, wqkv.compute, bqkv.master)  # [M, 3d]
            q5 = qkv.view(B, L, 3, heads, hd)
            o, lse = K.attn_fwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], kv_len, scale, causal)
            out = K.linear_fwd(o.view(B * L, d), wo.compute, bo.master)
            ctx.save_for_backward(x2, qkv, o, lse, kv_len)
            return out.view(B, L, d)
        qkv = x2 @ wqkv.master.t() + bqkv.master
        q5 = qkv.view(B, L, 3, heads, hd)
        o, pr = _ref_attn_fwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], kv_len, causal, scale)
        out = o.reshape(B * L, d) @ wo.master.t() + bo.master
        ctx.save_for_backward(x2, qkv, o, pr, kv_len)
        return out.view(B, L, d)

    @staticmethod
    def backward(ctx, dout):
        wqkv, bqkv, wo, bo = ctx.p
        heads, causal, scale, rt, fused_bo = ctx.meta
        x2, qkv, o, aux, kv_len = ctx.saved_tensors
        B, L, d = dout.shape
        M = B * L
        hd = d // heads
        dout2 = dout.reshape(M, d)
        beta = _beta(rt)
        if dout.is_cuda:
            dout2 = dout2.contiguous()
            o2 = o.view(M, d)
            K.linear_wgrad(dout2, o2, d, wo.grad, beta)
            if not fused_bo:
                K.colsum(dout2, d, bo.grad, beta)
            _ready(rt, wo, *([] if fused_bo else [bo]))
            do = K.linear_dgrad(dout2, wo.compute, d)
            dqkv = torch.empty(M, 3 * d, dtype=torch.bfloat16, device=dout.device)
            q5 = qkv.view(B, L, 3, heads, hd)
            g5 = dqkv.view(B, L, 3, heads, hd)
            K.attn_bwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o, do.view(B, L, heads, hd), aux,
                       g5[:, :, 0], g5[:, :, 1], g5[:, :, 2], kv_len, scale, causal)
            K.linear_wgrad(dqkv, x2, 3 * d, wqkv.grad, beta)
            K.colsum(dqkv, 3 * d, bqkv.grad, beta)
            _ready(rt, wqkv, bqkv)
            dx = K.linear_dgrad(dqkv, wqkv.compute, 3 * d)
            return dx.view(B, L, d), None, None, None, None, None, None, None, None, None
        o2 = o.reshape(M, d)
        _write_grad(wo, dout2.t() @ o2, rt)
        if not fused_bo:
            _write_grad(bo, dout2.sum(0), rt)
        do = (dout2 @ wo.master).view(B, L, heads, hd)
        q5 = qkv.view(B, L, 3, heads, hd)
        dq, dk, dv = _ref_attn_bwd(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], aux, do, scale)
        dqkv = torch.stack([dq, dk, dv], dim=2).reshape(M, 3 * d)
        _write_grad(wqkv, dqkv.t() @ x2, rt)
        _write_grad(bqkv, dqkv.sum(0), rt)
        _ready(rt, wo, *([] if fused_bo else [bo]), wqkv, bqkv)
        dx = dqkv @ wqkv.master
        return dx.view(B, L, d), None, None, None, None, None, None, None, None, None


class CrossMHAFn(torch.autograd.Function):
    """Decoder block 2: Q from the decoder stream, K = V = encoder output
    (reference call order mha2(enc, enc, out1) -> values, keys, query)."""

    @staticmethod
    def forward(ctx, x, enc, wq: Param, bq: Param, wkv: Param, bkv: Param, wo: Param, bo: Param,
                heads: int, kv_len, rt: RunCtx, fused_bo_grad: bool):
        B, T, d = x.shape
        S = enc.shape[1]
        hd = d // heads
        scale = 1.0 / math.sqrt(hd)
        ctx.p = (wq, bq, wkv, bkv, wo, bo)
        ctx.meta = (heads, scale, rt, fused_bo_grad)
        x2 = x.reshape(B * T, d)
        e2 = enc.reshape(B * S, d)
        if x.is_cuda:
            q = K.linear_fwd(x2, wq.compute, bq.master)
            kv = K.linear_fwd(e2, wkv.compute, bkv.master)
            kv5 = kv.view(B, S, 2, heads, hd)
            o, lse = K.attn_fwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], kv_len, scale,
                                False)
            out = K.linear_fwd(o.view(B * T, d), wo.compute, bo.master)
            ctx.save_for_backward(x2, e2, q, kv, o, lse, kv_len)
            return out.view(B, T, d)
        q = x2 @ wq.master.t() + bq.master
        kv = e2 @ wkv.master.t() + bkv.master
        kv5 = kv.view(B, S, 2, heads, hd)
        o, pr = _ref_attn_fwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], kv_len, False,
                              scale)
        out = o.reshape(B * T, d) @ wo.master.t() + bo.master
        ctx.save_for_backward(x2, e2, q, kv, o, pr, kv_len)
        return out.view(B, T, d)

    @staticmethod
    def backward(ctx, dout):
        wq, bq, wkv, bkv, wo, bo = ctx.p
        heads, scale, rt, fused_bo = ctx.meta
        x2, e2, q, kv, o, aux, kv_len = ctx.saved_tensors
        B, T, d = dout.shape
        S = e2.shape[0] // B
        hd = d // heads
        beta = _beta(rt)
        dout2 = dout.reshape(B * T, d)
        if dout.is_cuda:
            dout2 = dout2.contiguous()
            K.linear_wgrad(dout2, o.view(B * T, d), d, wo.grad, beta)
            if not fused_bo:
                K.colsum(dout2, d, bo.grad, beta)
            _ready(rt, wo, *([] if fused_bo else [bo]))
            do = K.linear_dgrad(dout2, wo.compute, d)
            dq = torch.empty(B * T, d, dtype=torch.bfloat16, device=dout.device)
            dkv = torch.empty(B * S, 2 * d, dtype=torch.bfloat16, device=dout.device)
            kv5 = kv.view(B, S, 2, heads, hd)
            g5 = dkv.view(B, S, 2, heads, hd)
            K.attn_bwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], o,
                       do.view(B, T, heads, hd), aux, dq.view(B, T, heads, hd), g5[:, :, 0],
                       g5[:, :, 1], kv_len, scale, False)
            K.linear_wgrad(dkv, e2, 2 * d, wkv.grad, beta)
            K.colsum(dkv, 2 * d, bkv.grad, beta)
            K.linear_wgrad(dq, x2, d, wq.grad, beta)
            K.colsum(dq, d, bq.grad, beta)
            _ready(rt, wkv, bkv, wq, bq)
            denc = K.linear_dgrad(dkv, wkv.compute, 2 * d)
            dx = K.linear_dgrad(dq, wq.compute, d)
            return (dx.view(B, T, d), denc.view(B, S, d)) + (None,) * 10
        o2 = o.reshape(B * T, d)
        _write_grad(wo, dout2.t() @ o2, rt)
        if not fused_bo:
            _write_grad(bo, dout2.sum(0), rt)
        do = (dout2 @ wo.master).view(B, T, heads, hd)
        kv5 = kv.view(B, S, 2, heads, hd)
        dqh, dk, dv = _ref_attn_bwd(q.view(B, T, heads, hd), kv5[:, :, 0], kv5[:, :, 1], aux, do,
                                    scale)
        dq = dqh.reshape(B * T, d)
        dkv = torch.stack([dk, dv], dim=2).reshape(B * S, 2 * d)
        _write_grad(wkv, dkv.t() @ e2, rt)
        _write_grad(bkv, dkv.sum(0), rt)
        _write_grad(wq, dq.t() @ x2, rt)
        _write_grad(bq, dq.sum(0), rt)
        _ready(rt, wo, *([] if fused_bo else [bo]), wkv, bkv, wq, bq)
        denc = dkv @ wkv.master
        dx = dq @ wq.master
        return (dx.view(B, T, d), denc.view(B, S, d)) + (None,) * 10


# =============================================================================== feed-forward
class FFNFn(torch.autograd.Function):
    """Dense(ff, relu) -> Dense(d); ReLU backward fused into the dgrad GEMM."""

    @staticmethod
    def forward(ctx, x, w1: Param, b1: Param, w2: Param, b2: Param, rt: RunCtx,
                fused_b2_grad: bool):
        B, L, d = x.shape
        x2 = x.reshape(B * L, d)
        ctx.p = (w1, b1, w2, b2)
        ctx.meta = (rt, fused_b2_grad)
        if x.is_cuda:
            h = K.linear_fwd(x2, w1.compute, b1.master, relu=True)
            y = K.linear_fwd(h, w2.compute, b2.master)
        else:
            h = torch.relu(x2 @ w1.master.t() + b1.master)
            y = h @ w2.master.t() + b2.master
        ctx.save_for_backward(x2, h)
        return y.view(B, L, d)

    @staticmethod
    def backward(ctx, dy):
        w1, b1, w2, b2 = ctx.p
        rt, fused_b2 = ctx.meta
        x2, h = ctx.saved_tensors
        B, L, d = dy.shape
        ff = h.shape[1]
        beta = _beta(rt)
        dy2 = dy.reshape(B * L, d)
        if dy.is_cuda:
            dy2 = dy2.contiguous()
            K.linear_wgrad(dy2, h, d, w2.grad, beta)
            if not fused_b2:
                K.colsum(dy2, d, b2.grad, beta)
            _ready(rt, w2, *([] if fused_b2 else [b2]))
            dpre = K.linear_dgrad(dy2, w2.compute, d, relu_aux=h)
            K.linear_wgrad(dpre, x2, ff, w1.grad, beta)
            K.colsum(dpre, ff, b1.grad, beta)
            _ready(rt, w1, b1)
            dx = K.linear_dgrad(dpre, w1.compute, ff)
            return dx.view(B, L, d), None, None, None, None, None, None
        _write_grad(w2, dy2.t() @ h, rt)
        if not fused_b2:
            _write_grad(b2, dy2.sum(0), rt)
        dpre = (dy2 @ w2.master) * (h > 0).to(dy2.dtype)
        _write_grad(w1, dpre.t() @ x2, rt)
        _write_grad(b1, dpre.sum(0), rt)
        _ready(rt, w2, *([] if fused_b2 else [b2]), w1, b1)
        dx = dpre @ w1.master
        return dx.view(B, L, d), None, None, None, None, None, None
