"""Independent plain-PyTorch f32 re-statement of the reference model's math
(reference: distributed_training_transformer/transformer_model.py), written
against TensorFlow variable names and the TF [in, out] kernel layout, with
end-to-end torch autograd. Used by the tests as the oracle for the fused
layer ops (forward values and every parameter gradient). Dropout is off.
"""
from __future__ import annotations

import math

import torch


def tf_weights(model) -> dict:
    """{tf_key: f64 tensor (requires_grad)} in TF layout, from a built model."""
    out = {}
    for p in model.store.params:
        for sl in p.tf:
            t = p.master.detach()[sl.row0:sl.row1]
            if sl.transpose:
                t = t.t()
            out[sl.key] = t.clone().double().requires_grad_(True)
    return out


def internal_grads_tf(model) -> dict:
    """The model's flat-buffer gradients re-expressed per TF key / layout."""
    out = {}
    for p in model.store.params:
        for sl in p.tf:
            g = p.grad.detach()[sl.row0:sl.row1]
            out[sl.key] = (g.t() if sl.transpose else g).double().cpu()
    return out


def _k(name):
    return name + "/.ATTRIBUTES/VARIABLE_VALUE"


def dense(W, prefix, x):
    return x @ W[_k(prefix + "/kernel")] + W[_k(prefix + "/bias")]


def layer_norm(W, prefix, x, eps=1e-6):
    mean = x.mean(-1, keepdim=True)
    var = ((x - mean) ** 2).mean(-1, keepdim=True)
    return (x - mean) / torch.sqrt(var + eps) * W[_k(prefix + "/gamma")] + W[_k(prefix + "/beta")]


def pos_encoding(L, d):
    pos = torch.arange(L, dtype=torch.float64).unsqueeze(1)
    i = torch.arange(d).unsqueeze(0)
    ang = pos / torch.pow(10000.0, (2 * (i // 2)).double() / d)
    return torch.where(i % 2 == 0, torch.sin(ang), torch.cos(ang))


def mha(W, prefix, v, k, q, mask, heads):
    B = q.shape[0]
    d = q.shape[-1]
    hd = d // heads
    Q = dense(W, prefix + "/query_generator_weights", q)
    Kk = dense(W, prefix + "/key_generator_weights", k)
    V = dense(W, prefix + "/value_generator_weights", v)

    def split(x):
        return x.view(B, -1, heads, hd).transpose(1, 2)

    Q, Kk, V = split(Q), split(Kk), split(V)
    logits = Q @ Kk.transpose(-1, -2) / math.sqrt(hd)
    # the mask add happens in fp32 as in TF (a fully masked row's logits all
    # round to -1e9: uniform softmax); autograd passes the gradient through
    logits = (logits.float() + (mask * -1e9).float()).double()
    w = torch.softmax(logits, -1)
    o = (w @ V).transpose(1, 2).reshape(B, -1, d)
    return dense(W, prefix + "/dense", o), w


def ffn(W, prefix, x):
    h = torch.relu(dense(W, prefix + "/layer_with_weights-0", x))
    return dense(W, prefix + "/layer_with_weights-1", h)


def forward(W, src, tgt_in, cfg):
    d, heads, L = cfg.d_model, cfg.heads, cfg.layers
    enc_pad = (src == 0).double()[:, None, None, :]
    T = tgt_in.shape[1]
    look = 1 - torch.tril(torch.ones(T, T, dtype=torch.float64))
    look = torch.maximum((tgt_in == 0).double()[:, None, None, :], look)
    x = W[_k("encoder/embedding/embeddings")][src] * math.sqrt(d) + pos_encoding(src.shape[1], d)
    for i in range(L):
        p = f"encoder/encoder_layers/{i}"
        a, _ = mha(W, p + "/mha", x, x, x, enc_pad, heads)
        x = layer_norm(W, p + "/layernorm1", x + a)
        x = layer_norm(W, p + "/layernorm2", x + ffn(W, p + "/ffn", x))
    enc = x
    y = W[_k("decoder/embedding/embeddings")][tgt_in] * math.sqrt(d) + pos_encoding(T, d)
    for i in range(L):
        p = f"decoder/decoder_layers/{i}"
        a, _ = mha(W, p + "/mha1", y, y, y, look, heads)
        y = layer_norm(W, p + "/layernorm1", a + y)
        c, _ = mha(W, p + "/mha2", enc, enc, y, enc_pad, heads)
        y = layer_norm(W, p + "/layernorm2", c + y)
        y = layer_norm(W, p + "/layernorm3", ffn(W, p + "/ffn", y) + y)
    return dense(W, "final_layer", y)


def loss_fn(W, src, tgt, cfg, workers=1.0):
    tgt_in, real = tgt[:, :-1], tgt[:, 1:]
    logits = forward(W, src, tgt_in, cfg)
    mask = (real != 0).double()
    ce = torch.nn.functional.cross_entropy(logits.reshape(-1, logits.shape[-1]), real.reshape(-1),
                                           reduction="none").view_as(mask)
    loss = (ce * mask).sum() / mask.sum() / workers
    acc = (((logits.argmax(-1) == real).double() * mask).sum() / mask.sum())
    return loss, acc, logits
