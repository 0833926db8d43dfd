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

from tensorflow_distributed_on_gke_amd.models.layers import CrossKVFn, EmbedFn, KVGrad, RunCtx
from tensorflow_distributed_on_gke_amd.models.transformer import PAD_ID, Transformer, seq_lengths
from tensorflow_distributed_on_gke_amd.ops import kernels as K


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
    def attention_weights(self, src: torch.Tensor, tgt_in: torch.Tensor) -> Dict[str, torch.Tensor]:
        m = self.model
        rt = RunCtx(training=False, store=None, attn_maps={})
        m.features(src.to(m.device), tgt_in.to(m.device), rt)
        out = {}
        for i, layer in enumerate(m.dec_layers):
            out[f"decoder_layer{i + 1}_block1"] = rt.attn_maps[layer.site1]
            out[f"decoder_layer{i + 1}_block2"] = rt.attn_maps[layer.site2]
        return out

    def __call__(self, sentence: Union[str, Sequence[str]], max_length: int = 20
                 ) -> Tuple[Union[str, List[str]], list, Dict[str, torch.Tensor]]:
        single = isinstance(sentence, str)
        src = self.src_tok.tokenize(sentence)
        out = self.greedy(src, max_length).cpu()
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
