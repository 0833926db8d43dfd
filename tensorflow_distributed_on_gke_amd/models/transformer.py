"""Encoder-decoder Transformer (post-LN, "Attention Is All You Need" / the TF
Transformer tutorial), built on the fused gfx950 layer ops.

Reference model: distributed_training_transformer/transformer_model.py
(Transformer :318-348, masks :350-363, TransformerEncoder :251-279,
TransformerDecoder :282-315, EncoderLayer :178-204, DecoderLayer :207-248,
positional_encoding :29-53, loss :11-17, accuracy :20-26).

Parameters are registered under the reference's TensorFlow variable names so
checkpoints interchange with `model.save_weights` bundles;
internal layouts are GPU-friendly ([out, in] weights, fused QKV / KV) and the
TensorBundle I/O maps them back to the reference's separate [in, out] Dense
kernels.
"""
from __future__ import annotations

import math
from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from tensorflow_distributed_on_gke_amd.models.layers import (_dgrad_res, _wgrad,
                                                              CrossAttnBlockFn, CrossKVFn, EmbedFn,
                                                              FFNBlockFn, KVGrad, RunCtx,
                                                              SelfAttnBlockFn)
from tensorflow_distributed_on_gke_amd.models.params import (ParamStore, TFSlot, const,
                                                              glorot_blocks, glorot_uniform,
                                                              uniform)
from tensorflow_distributed_on_gke_amd.ops import kernels as K

PAD_ID = 0


@dataclass
class ModelConfig:
    layers: int = 4
    d_model: int = 128
    heads: int = 8
    d_ff: int = 512
    src_vocab: int = 7765
    tgt_vocab: int = 7010
    max_src_len: int = 1000
    max_tgt_len: int = 1000
    dropout: float = 0.1
    label_smoothing: float = 0.0

    def to_dict(self) -> dict:
        return asdict(self)


# BASELINE.json configs. "reference" = the reference's hard-coded model
# (reference: distributed_training_transformer/__main__.py:39-43; vocab sizes
# decoded from saved_weights/2/model_weights.index).
PRESETS: Dict[str, dict] = {
    "reference": dict(layers=4, d_model=128, heads=8, d_ff=512),
    "tiny": dict(layers=2, d_model=128, heads=8, d_ff=512),
    "base": dict(layers=6, d_model=512, heads=8, d_ff=2048),
    "big": dict(layers=6, d_model=1024, heads=16, d_ff=4096),
}


def model_config(preset: str = "reference", **over) -> ModelConfig:
    if preset not in PRESETS:
        raise KeyError(f"unknown preset {preset!r}; have {sorted(PRESETS)}")
    kw = dict(PRESETS[preset])
    kw.update({k: v for k, v in over.items() if v is not None})
    return ModelConfig(**kw)


def positional_encoding(length: int, d: int) -> torch.Tensor:
    """[length, d] f32, sin on even dims / cos on odd dims (interleaved), angle
    = pos / 10000^(2*(i//2)/d), computed in f32 like the reference."""
    pos = torch.arange(length, dtype=torch.float32).unsqueeze(1)
    i = torch.arange(d).unsqueeze(0)
    rates = 1.0 / torch.pow(torch.tensor(10000.0), (2 * (i // 2)).to(torch.float32) / float(d))
    ang = pos * rates
    return torch.where(i % 2 == 0, torch.sin(ang), torch.cos(ang)).to(torch.float32)


def _var(key: str) -> str:
    return key + "/.ATTRIBUTES/VARIABLE_VALUE"


class _Dense:
    """Registers a Dense layer, or a fused stack of several Dense layers that
    read the same input (their [out, in] kernels stacked along `out`)."""

    def __init__(self, store: ParamStore, name: str, tf_prefixes: List[str], d_in: int, d_out: int):
        k = len(tf_prefixes)
        wslots = [TFSlot(_var(p + "/kernel"), i * d_out, (i + 1) * d_out, True)
                  for i, p in enumerate(tf_prefixes)]
        bslots = [TFSlot(_var(p + "/bias"), i * d_out, (i + 1) * d_out, False)
                  for i, p in enumerate(tf_prefixes)]
        self.w = store.add(name + "/kernel", (k * d_out, d_in), glorot_blocks(d_out, d_in, d_out),
                           wslots)
        self.b = store.add(name + "/bias", (k * d_out,), const(0.0), bslots)


class _LN:
    def __init__(self, store: ParamStore, prefix: str, d: int):
        self.gamma = store.add(prefix + "/gamma", (d,), const(1.0), [TFSlot(_var(prefix + "/gamma"), 0, d, False)])
        self.beta = store.add(prefix + "/beta", (d,), const(0.0), [TFSlot(_var(prefix + "/beta"), 0, d, False)])


class EncoderLayer:
    """reference: transformer_model.py:178-204"""

    def __init__(self, store: ParamStore, i: int, cfg: ModelConfig, sites):
        d, ff = cfg.d_model, cfg.d_ff
        pre = f"encoder/encoder_layers/{i}"
        m = pre + "/mha"
        self.qkv = _Dense(store, m + "/qkv", [m + "/query_generator_weights", m + "/key_generator_weights",
                                              m + "/value_generator_weights"], d, d)
        self.o = _Dense(store, m + "/dense", [m + "/dense"], d, d)
        self.ln1 = _LN(store, pre + "/layernorm1", d)
        self.ff1 = _Dense(store, pre + "/ffn/layer_with_weights-0", [pre + "/ffn/layer_with_weights-0"], d, ff)
        self.ff2 = _Dense(store, pre + "/ffn/layer_with_weights-1", [pre + "/ffn/layer_with_weights-1"], ff, d)
        self.ln2 = _LN(store, pre + "/layernorm2", d)
        self.site1, self.site2 = next(sites), next(sites)
        self.heads = cfg.heads

    def __call__(self, x, src_len, rt: RunCtx):
        x = SelfAttnBlockFn.apply(x, self.qkv.w, self.qkv.b, self.o.w, self.o.b, self.ln1.gamma,
                                  self.ln1.beta, self.heads, src_len, False, self.site1, rt)
        return FFNBlockFn.apply(x, self.ff1.w, self.ff1.b, self.ff2.w, self.ff2.b, self.ln2.gamma,
                                self.ln2.beta, self.site2, rt)


class DecoderLayer:
    """reference: transformer_model.py:207-248 (the cross-attention K/V
    projections of all layers live in Transformer.cross_kv)"""

    def __init__(self, store: ParamStore, i: int, cfg: ModelConfig, sites):
        d, ff = cfg.d_model, cfg.d_ff
        pre = f"decoder/decoder_layers/{i}"
        m1, m2 = pre + "/mha1", pre + "/mha2"
        self.index = i
        self.qkv1 = _Dense(store, m1 + "/qkv", [m1 + "/query_generator_weights", m1 + "/key_generator_weights",
                                                m1 + "/value_generator_weights"], d, d)
        self.o1 = _Dense(store, m1 + "/dense", [m1 + "/dense"], d, d)
        self.ln1 = _LN(store, pre + "/layernorm1", d)
        self.q2 = _Dense(store, m2 + "/query_generator_weights", [m2 + "/query_generator_weights"], d, d)
        self.o2 = _Dense(store, m2 + "/dense", [m2 + "/dense"], d, d)
        self.ln2 = _LN(store, pre + "/layernorm2", d)
        self.ff1 = _Dense(store, pre + "/ffn/layer_with_weights-0", [pre + "/ffn/layer_with_weights-0"], d, ff)
        self.ff2 = _Dense(store, pre + "/ffn/layer_with_weights-1", [pre + "/ffn/layer_with_weights-1"], ff, d)
        self.ln3 = _LN(store, pre + "/layernorm3", d)
        self.site1, self.site2, self.site3 = next(sites), next(sites), next(sites)
        self.heads = cfg.heads

    def __call__(self, x, kv_all, kvh: KVGrad, src_len, tgt_len, rt: RunCtx):
        x = SelfAttnBlockFn.apply(x, self.qkv1.w, self.qkv1.b, self.o1.w, self.o1.b, self.ln1.gamma,
                                  self.ln1.beta, self.heads, tgt_len, True, self.site1, rt)
        x = CrossAttnBlockFn.apply(x, kv_all, self.index, kvh, self.q2.w, self.q2.b, self.o2.w,
                                   self.o2.b, self.ln2.gamma, self.ln2.beta, self.heads, src_len,
                                   self.site2, rt)
        return FFNBlockFn.apply(x, self.ff1.w, self.ff1.b, self.ff2.w, self.ff2.b, self.ln3.gamma,
                                self.ln3.beta, self.site3, rt)


TRANSPOSED_FFN_DGRAD = True
# smallest d_model that keeps W2^T for the FFN relu-backward dgrad
TRANSPOSED_FFN_MIN_D = 1024


def seq_lengths(tok: torch.Tensor, check: bool = True) -> torch.Tensor:
    """Valid (non-PAD) length per row for right-padded batches -> int32 [B]
    (the reference's padding mask `tok == 0`, transformer_model.py:56-62).
    Attention masks keys by this length, so a PAD before a non-PAD token
    (which the reference would mask individually) is rejected: on the CPU
    here (`check`), on the GPU by the batch-prep kernel's bad-row counter
    (ops.kernels.check_trailing_padding)."""
    nz = tok != PAD_ID
    n = nz.sum(dim=1, dtype=torch.int32)
    if check and tok.device.type == "cpu" and tok.numel():
        pos = torch.arange(1, tok.shape[1] + 1, dtype=torch.int32).expand_as(tok)
        last = torch.where(nz, pos, torch.zeros_like(pos)).amax(dim=1)
        if not torch.equal(last, n):
            raise ValueError("sequences must be right-padded: a PAD (id 0) token precedes a "
                             "non-PAD token (attention masks keys by length)")
    return n


class Transformer:
    def __init__(self, cfg: ModelConfig, store: Optional[ParamStore] = None):
        if cfg.d_model % cfg.heads:
            raise ValueError("d_model must be divisible by heads")
        self.cfg = cfg
        self.store = store or ParamStore()
        S = self.store
        d = cfg.d_model
        sites = iter(range(1, 4096))
        # forward order of registration (flat layout is the reverse; see params.py)
        self.enc_emb = S.add("encoder/embedding/embeddings", (cfg.src_vocab, d), uniform(-0.05, 0.05),
                             [TFSlot(_var("encoder/embedding/embeddings"), 0, cfg.src_vocab, False)])
        self.enc_site = next(sites)
        self.enc_layers = [EncoderLayer(S, i, cfg, sites) for i in range(cfg.layers)]
        # K|V projections of the encoder output for every decoder layer,
        # stacked [layers*2*d, d] so the forward is one GEMM (reference: each
        # decoder_layers/{i}/mha2/{key,value}_generator_weights Dense)
        kv_prefixes = []
        for i in range(cfg.layers):
            m2 = f"decoder/decoder_layers/{i}/mha2"
            kv_prefixes += [m2 + "/key_generator_weights", m2 + "/value_generator_weights"]
        self.cross_kv = _Dense(S, "decoder/cross_kv_all", kv_prefixes, d, d)
        self.dec_emb = S.add("decoder/embedding/embeddings", (cfg.tgt_vocab, d), uniform(-0.05, 0.05),
                             [TFSlot(_var("decoder/embedding/embeddings"), 0, cfg.tgt_vocab, False)])
        self.dec_site = next(sites)
        self.dec_layers = [DecoderLayer(S, i, cfg, sites) for i in range(cfg.layers)]
        self.final = _Dense(S, "final_layer", ["final_layer"], d, cfg.tgt_vocab)
        self.vocab_pad = (cfg.tgt_vocab + 63) // 64 * 64
        self.pe_src: Optional[torch.Tensor] = None
        self.pe_tgt: Optional[torch.Tensor] = None
        self.device = torch.device("cpu")

    # ------------------------------------------------------------------ setup
    def build(self, device="cpu", seed: int = 0, compute_dtype=torch.bfloat16) -> "Transformer":
        self.device = torch.device(device)
        self.store.finalize(self.device, compute_dtype, seed)
        if self.device.type == "cuda" and TRANSPOSED_FFN_DGRAD and self.cfg.d_model >= TRANSPOSED_FFN_MIN_D:
            # the FFN's relu-backward dgrad reads W2 K-contiguous the other way
            # round: keep W2^T so it runs with the forward-layout (NT) 256x256
            # kernel. Measured per call: d 1024 / ff 4096: 111.5 -> 102.6 us
            # (NN 128x128 vs NT 256x256); d 512 / ff 2048: NN 64x128 39.7 us
            # beats NT 43.0 us, so Transformer-base keeps the NN dgrad.
            for layer in self.enc_layers + self.dec_layers:
                self.store.add_transposed(layer.ff2.w)
        self.pe_src = positional_encoding(self.cfg.max_src_len, self.cfg.d_model).to(self.device)
        self.pe_tgt = positional_encoding(self.cfg.max_tgt_len, self.cfg.d_model).to(self.device)
        return self

    @property
    def act_dtype(self):
        return torch.bfloat16 if self.device.type == "cuda" else torch.float32

    def num_params(self) -> int:
        return self.store.num_params()

    # ------------------------------------------------------------------ forward
    def encode(self, src: torch.Tensor, src_len: torch.Tensor, rt: RunCtx) -> torch.Tensor:
        if src.shape[1] > self.cfg.max_src_len:
            raise ValueError(f"source length {src.shape[1]} > positional table {self.cfg.max_src_len}")
        x = EmbedFn.apply(self.store.anchor, src.contiguous(), self.enc_emb, self.pe_src, self.enc_site, rt)
        for layer in self.enc_layers:
            x = layer(x, src_len, rt)
        return x

    def decode(self, tgt_in: torch.Tensor, enc: torch.Tensor, src_len, tgt_len, rt: RunCtx) -> torch.Tensor:
        if tgt_in.shape[1] > self.cfg.max_tgt_len:
            raise ValueError(f"target length {tgt_in.shape[1]} > positional table {self.cfg.max_tgt_len}")
        kvh = KVGrad()
        kvh.dec_len, kvh.heads, kvh.wkv = tgt_in.shape[1], self.cfg.heads, self.cross_kv.w
        kv_all = CrossKVFn.apply(enc, self.cross_kv.w, self.cross_kv.b, kvh, rt)
        x = EmbedFn.apply(self.store.anchor, tgt_in.contiguous(), self.dec_emb, self.pe_tgt, self.dec_site, rt)
        try:
            for layer in self.dec_layers:
                x = layer(x, kv_all, kvh, src_len, tgt_len, rt)
        finally:
            if rt.fp8 is not None:
                rt.fp8.kv8 = None  # this forward's e4m3 K|V: never seen by the next one
        return x

    def features(self, src, tgt_in, rt: RunCtx, lengths=None):
        src_len, tgt_len = lengths if lengths is not None else (seq_lengths(src), seq_lengths(tgt_in))
        rt.emb_csr = None
        if (src.is_cuda and rt.training and torch.is_grad_enabled()
                and K.embed_csr_ok(src.numel(), self.cfg.src_vocab)
                and K.embed_csr_ok(tgt_in.numel(), self.cfg.tgt_vocab)):
            # both embedding backwards' token sorts in one launch, now: the
            # tokens are known (ops.kernels.EmbCsr)
            cs = K.embed_csr_sort([(src, self.enc_emb.shape[0], "enc"),
                                   (tgt_in, self.dec_emb.shape[0], "dec")])
            rt.emb_csr = {self.enc_site: cs[0], self.dec_site: cs[1]}
        enc = self.encode(src, src_len, rt)
        return self.decode(tgt_in, enc, src_len, tgt_len, rt)

    def project(self, dec: torch.Tensor) -> torch.Tensor:
        """Final Dense -> logits. GPU: bf16 [B*T, vocab_pad] (padded row);
        CPU: f32 [B*T, vocab]."""
        B, T, d = dec.shape
        d2 = dec.reshape(B * T, d)
        if dec.is_cuda:
            return K.linear_fwd(d2.contiguous(), self.final.w.compute, self.final.b.master,
                                ldc=self.vocab_pad)
        return d2 @ self.final.w.master.t() + self.final.b.master

    def logits(self, src, tgt_in, rt: Optional[RunCtx] = None) -> torch.Tensor:
        """[B, T, V] f32 logits (inference / tests)."""
        rt = rt or RunCtx(training=False, store=None)
        with torch.no_grad():
            dec = self.features(src, tgt_in, rt)
            lg = self.project(dec)
        B, T = tgt_in.shape
        return lg[:, : self.cfg.tgt_vocab].float().reshape(B, T, self.cfg.tgt_vocab)

    # ------------------------------------------------------------------ training
    def loss_and_backward(self, src, tgt, rt: RunCtx, workers: float,
                          accum: Optional[torch.Tensor] = None, backward: bool = True,
                          step_out: Optional[torch.Tensor] = None,
                          bump_ctr: bool = False, ntok_sum=None) -> torch.Tensor:
        """Teacher-forced forward, masked CE / accuracy, and (if `backward`)
        the full backward into the flat gradient buffer. Returns a device
        tensor [local_loss, accuracy] (loss already / workers, as the
        reference's local_loss_function). No host synchronisation.
        bump_ctr: advance the dropout RNG step counter rt.ctr first.
        ntok_sum: global-token-mean loss -- called with this replica's label
        count, turns it in place into the count over all replicas (returns an
        async work handle or None); pass workers = 1 with it."""
        cfg = self.cfg
        dev = src.device
        if dev.type == "cuda":  # split / lengths / token count / ctr: one launch
            tgt_in, labels, src_len, tgt_len, ntok = K.prep_batch(
                src, tgt, rt.ctr if bump_ctr else None)
            lengths = (src_len, tgt_len)
            # the label count all-reduce flies during the forward
            ntok_work = ntok_sum(ntok) if ntok_sum is not None else None
        else:
            if bump_ctr:
                rt.ctr.add_(1)
            tgt_in = tgt[:, :-1].contiguous()
            labels = tgt[:, 1:].contiguous()
            lengths = None
        B, T = tgt_in.shape
        M = B * T
        if step_out is None:
            step_out = torch.zeros(2, dtype=torch.float32, device=dev)
        grad_ctx = torch.enable_grad() if backward else torch.no_grad()
        with grad_ctx:
            dec = self.features(src, tgt_in, rt, lengths)
        dec2 = dec.detach().reshape(M, cfg.d_model)
        if dev.type == "cuda":
            logits = self.project(dec.detach())
            row_loss = K.workspace("row_loss", M, dev)[:M]
            row_cor = K.workspace("row_correct", M, dev)[:M]
            if ntok_work is not None:
                ntok_work.wait()
            K.xent(logits, cfg.tgt_vocab, labels, ntok, workers, cfg.label_smoothing, row_loss,
                   row_cor, write_grad=backward)
            K.xent_stats(row_loss, row_cor, ntok, workers, step_out, accum)
            if not backward:
                return step_out
            beta = 1.0 if rt.accumulate else 0.0
            dl = logits  # now holds dlogits (pad columns zeroed)
            _wgrad(rt, dl, dec2.contiguous(), cfg.tgt_vocab, self.final.w, self.final.b)
            ddec = _dgrad_res(dl, self.final.w, cfg.tgt_vocab, None)
        else:
            lg = self.project(dec.detach())
            lab = labels.reshape(-1)
            mask = (lab != PAD_ID).to(torch.float32)
            ntok = mask.sum()
            if ntok_sum is not None:
                w = ntok_sum(ntok)
                if w is not None:
                    w.wait()
            ntok = ntok.clamp_min(1.0)
            logp = torch.log_softmax(lg, dim=-1)
            eps = cfg.label_smoothing
            nll = -logp.gather(1, lab.view(-1, 1)).squeeze(1)
            smooth = -logp.mean(dim=-1)
            row_loss = ((1 - eps) * nll + eps * smooth) * mask
            correct = ((lg.argmax(dim=-1) == lab).to(torch.float32) * mask).sum()
            loss = row_loss.sum() / ntok / workers
            acc = correct / ntok
            step_out.copy_(torch.stack([loss, acc]).detach())
            if accum is not None:
                accum += torch.stack([loss.detach(), acc.detach(), torch.tensor(1.0), ntok])
            if not backward:
                return step_out
            onehot = torch.nn.functional.one_hot(lab, cfg.tgt_vocab).to(torch.float32)
            dl = (torch.softmax(lg, -1) - (1 - eps) * onehot - eps / cfg.tgt_vocab)
            dl = dl * (mask / (ntok * workers)).view(-1, 1)
            fw, fb = self.final.w, self.final.b
            g_w = dl.t() @ dec2
            g_b = dl.sum(0)
            if rt.accumulate:
                fw.grad.add_(g_w)
                fb.grad.add_(g_b)
            else:
                fw.grad.copy_(g_w)
                fb.grad.copy_(g_b)
            if rt.store is not None:
                rt.store.grad_ready(fw)
                rt.store.grad_ready(fb)
            ddec = dl @ fw.master
        dec.backward(ddec.view(B, T, cfg.d_model).to(dec.dtype))
        if rt.wgrad is not None:
            rt.wgrad.flush()
            rt.wgrad.step_done()
        return step_out
