"""Greedy translation harness (reference: distributed_training_transformer/
tester.py:4-59 and test.py:1-44).

Same contract as the reference Tester: tokenize the source, start the target
with [START], append the argmax token until [END] or `max_length`, return
(text, tokens, attention_weights), where the attention weights are recomputed
on output[:, :-1] and keyed `decoder_layer{i}_block{1,2}` [B, H, Lq, Lk].

MI355X design: batched (many sentences decode together; finished rows are
padded), the encoder output and the stacked cross-attention K/V projection
are computed once per call instead of once per generated token, and each
step runs the decoder stack through the same HIP kernels as training, with
only the last position projected to the vocabulary.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple, Union

import torch

from tensorflow_distributed_on_gke_amd.models.layers import (LN_EPS, CrossKVFn, EmbedFn, KVGrad,
                                                             RunCtx, _ref_attn_fwd)
from tensorflow_distributed_on_gke_amd.models.transformer import PAD_ID, Transformer, seq_lengths
from tensorflow_distributed_on_gke_amd.ops import kernels as K


# --------------------------------------------------------------- single-token ops (GPU kernels / CPU f32)
def _linear(x2, dense, relu=False):
    if x2.is_cuda:
        return K.linear_fwd(x2.contiguous(), dense.w.compute, dense.b.master, relu=relu)
    y = x2 @ dense.w.master.t() + dense.b.master
    return torch.relu(y) if relu else y


def _add_ln(x, s, ln):
    if x.is_cuda:
        return K.ln_fwd(x.contiguous(), s.contiguous(), ln.gamma.master, ln.beta.master, 0.0, 0, None, 0,
                        save=False)[0]
    return torch.nn.functional.layer_norm(x + s, (x.shape[-1],), ln.gamma.master, ln.beta.master, LN_EPS)


def _attend(q, k, v, kv_len, scale):
    if q.is_cuda:
        return K.attn_fwd(q, k, v, kv_len, scale, False)[0]
    return _ref_attn_fwd(q, k, v, kv_len, False, scale)[0]


class Tester:
    __test__ = False  # not a pytest class

    def __init__(self, tokenizers, transformer: Transformer):
        """`tokenizers` has `.pt` (source) and `.en` (target) tokenizers, as
        the reference's; a single tokenizer object is used for both."""
        self.src_tok = getattr(tokenizers, "pt", tokenizers)
        self.tgt_tok = getattr(tokenizers, "en", tokenizers)
        self.model = transformer

    @torch.no_grad()
    def greedy(self, src: torch.Tensor, max_length: int = 20) -> torch.Tensor:
        """src int64 [B, S] -> int64 [B, 1 + n] ([START] + generated ids)."""
        m = self.model
        dev = m.device
        src = src.to(dev)
        start, end = self.tgt_tok.start_end()
        B = src.shape[0]
        rt = RunCtx(training=False, store=None)
        src_len = seq_lengths(src)
        enc = m.encode(src, src_len, rt)
        kv_all = CrossKVFn.apply(enc, m.cross_kv.w, m.cross_kv.b, KVGrad(), rt)
        out = torch.full((B, 1), start, dtype=torch.int64, device=dev)
        done = torch.zeros(B, dtype=torch.bool, device=dev)
        for _ in range(max_length):
            tgt_len = seq_lengths(out)
            x = EmbedFn.apply(m.store.anchor, out, m.dec_emb, m.pe_tgt, m.dec_site, rt)
            kvh = KVGrad()
            for layer in m.dec_layers:
                x = layer(x, kv_all, kvh, src_len, tgt_len, rt)
            last = x[:, -1:, :]
            lg = m.project(last.contiguous())[:, : m.cfg.tgt_vocab].float()
            nxt = lg.argmax(dim=-1)
            nxt = torch.where(done, torch.full_like(nxt, PAD_ID), nxt)
            out = torch.cat([out, nxt.view(B, 1)], dim=1)
            done |= nxt == end
            if bool(done.all()):
                break
        return out

    @torch.no_grad()
    def greedy_cached(self, src: torch.Tensor, max_length: int = 20) -> torch.Tensor:
        """Greedy decoding with a per-layer self-attention K/V cache: each step
        runs the decoder on the ONE new token (O(T) work per step instead of
        the reference's full re-forward, tester.py:30-42). Same output as
        `greedy` up to floating-point summation order."""
        m = self.model
        cfg = m.cfg
        dev = m.device
        src = src.to(dev)
        start, end = self.tgt_tok.start_end()
        B = src.shape[0]
        d, H = cfg.d_model, cfg.heads
        hd = d // H
        scale = 1.0 / (hd ** 0.5)
        rt = RunCtx(training=False, store=None)
        src_len = seq_lengths(src)
        enc = m.encode(src, src_len, rt)
        S = enc.shape[1]
        kv_all = CrossKVFn.apply(enc, m.cross_kv.w, m.cross_kv.b, KVGrad(), rt).contiguous()
        act = m.act_dtype
        Tm = max_length + 1
        kcache = [torch.zeros(B, Tm, H, hd, dtype=act, device=dev) for _ in m.dec_layers]
        vcache = [torch.zeros(B, Tm, H, hd, dtype=act, device=dev) for _ in m.dec_layers]
        out = torch.full((B, 1), start, dtype=torch.int64, device=dev)
        done = torch.zeros(B, dtype=torch.bool, device=dev)
        for t in range(max_length):
            tok = out[:, -1:]
            if dev.type == "cuda":
                x = K.embed_fwd(tok.contiguous(), m.dec_emb.compute, m.pe_tgt[t:], d ** 0.5, 0.0, 0,
                                None, 0)
            else:
                x = m.dec_emb.master[tok] * (d ** 0.5) + m.pe_tgt[t].view(1, 1, d)
            x2 = x.reshape(B, d)
            klen = torch.full((B,), t + 1, dtype=torch.int32, device=dev)
            for li, layer in enumerate(m.dec_layers):
                qkv = _linear(x2, layer.qkv1).view(B, 1, 3, H, hd)
                kcache[li][:, t] = qkv[:, 0, 1]
                vcache[li][:, t] = qkv[:, 0, 2]
                o = _attend(qkv[:, :, 0], kcache[li][:, : t + 1], vcache[li][:, : t + 1], klen, scale)
                y = _add_ln(x2, _linear(o.reshape(B, d), layer.o1), layer.ln1)
                q2 = _linear(y, layer.q2).view(B, 1, H, hd)
                kv5 = kv_all[:, :, li * 2 * d:(li + 1) * 2 * d].view(B, S, 2, H, hd)
                o2 = _attend(q2, kv5[:, :, 0], kv5[:, :, 1], src_len, scale)
                y2 = _add_ln(y, _linear(o2.reshape(B, d), layer.o2), layer.ln2)
                f = _linear(_linear(y2, layer.ff1, relu=True), layer.ff2)
                x2 = _add_ln(y2, f, layer.ln3)
            lg = m.project(x2.view(B, 1, d))[:, : cfg.tgt_vocab].float()
            nxt = lg.argmax(dim=-1)
            nxt = torch.where(done, torch.full_like(nxt, PAD_ID), nxt)
            out = torch.cat([out, nxt.view(B, 1)], dim=1)
            done |= nxt == end
            if bool(done.all()):
                break
        return out

    @torch.no_grad()
    def attention_weights(self, src: torch.Tensor, tgt_in: torch.Tensor) -> Dict[str, torch.Tensor]:
        m = self.model
        rt = RunCtx(training=False, store=None, attn_maps={})
        m.features(src.to(m.device), tgt_in.to(m.device), rt)
        out = {}
        for i, layer in enumerate(m.dec_layers):
            out[f"decoder_layer{i + 1}_block1"] = rt.attn_maps[layer.site1]
            out[f"decoder_layer{i + 1}_block2"] = rt.attn_maps[layer.site2]
        return out

    def __call__(self, sentence: Union[str, Sequence[str]], max_length: int = 20, kv_cache: bool = True
                 ) -> Tuple[Union[str, List[str]], list, Dict[str, torch.Tensor]]:
        single = isinstance(sentence, str)
        src = self.src_tok.tokenize(sentence)
        out = (self.greedy_cached if kv_cache else self.greedy)(src, max_length).cpu()
        texts, tokens = [], []
        _, end = self.tgt_tok.start_end()
        for row in out.tolist():
            if end in row:
                row = row[: row.index(end) + 1]
            row = [t for t in row if t != PAD_ID]
            texts.append(self.tgt_tok.detokenize(row))
            tokens.append(self.tgt_tok.lookup(row))
        attn = self.attention_weights(src, out[:, :-1])
        if single:
            return texts[0], tokens[0], attn
        return texts, tokens, attn
