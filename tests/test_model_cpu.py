"""CPU tests of the fused layer ops against an independent autograd oracle."""
import pytest
import torch

import ref_model
from tensorflow_distributed_on_gke_amd.models.layers import RunCtx
from tensorflow_distributed_on_gke_amd.models.transformer import (Transformer, model_config,
                                                                  positional_encoding)


def _batch(B, S, T, V1, V2, seed=0, pad=True):
    g = torch.Generator().manual_seed(seed)
    src = torch.randint(4, V1, (B, S), generator=g)
    tgt = torch.randint(4, V2, (B, T), generator=g)
    if pad:
        for b in range(B):
            ls = int(torch.randint(3, S + 1, (1,), generator=g))
            lt = int(torch.randint(3, T + 1, (1,), generator=g))
            src[b, ls:] = 0
            tgt[b, lt:] = 0
    return src, tgt


def test_reference_param_count():
    # 4,646,882 parameters in 172 TF variables
    m = Transformer(model_config("reference"))
    assert m.num_params() == 4646882
    keys = [s.key for p in m.store.params for s in p.tf]
    assert len(keys) == 172 and len(set(keys)) == 172


@pytest.mark.parametrize("preset,expect", [("base", 55299426), ("big", 198672226)])
def test_preset_param_counts(preset, expect):
    assert Transformer(model_config(preset)).num_params() == expect


def test_positional_encoding_interleaved():
    pe = positional_encoding(50, 16)
    import math
    for pos in (0, 7, 49):
        for i in range(16):
            ang = pos / (10000 ** ((2 * (i // 2)) / 16))
            ref = math.sin(ang) if i % 2 == 0 else math.cos(ang)
            assert abs(pe[pos, i].item() - ref) < 1e-5


@pytest.mark.parametrize("workers", [1.0, 3.0])
def test_forward_backward_matches_oracle(workers):
    cfg = model_config("tiny", d_model=32, heads=4, d_ff=64, src_vocab=50, tgt_vocab=40, dropout=0.0)
    m = Transformer(cfg).build("cpu", seed=3)
    src, tgt = _batch(3, 9, 8, 50, 40, seed=1)
    rt = RunCtx(training=True, dropout=0.0, store=m.store)
    out = m.loss_and_backward(src, tgt, rt, workers=workers)
    W = ref_model.tf_weights(m)
    loss, acc, _ = ref_model.loss_fn(W, src, tgt, cfg, workers)
    loss.backward()
    assert abs(out[0].item() - loss.item()) < 1e-5
    assert abs(out[1].item() - acc.item()) < 1e-6
    ours = ref_model.internal_grads_tf(m)
    assert set(ours) == set(W)
    for k, t in W.items():
        torch.testing.assert_close(ours[k], t.grad, rtol=2e-4, atol=2e-6, msg=k)


def test_logits_match_oracle():
    cfg = model_config("tiny", d_model=32, heads=4, d_ff=64, src_vocab=50, tgt_vocab=40)
    m = Transformer(cfg).build("cpu", seed=4)
    src, tgt = _batch(2, 7, 6, 50, 40, seed=2)
    lg = m.logits(src, tgt[:, :-1])
    W = ref_model.tf_weights(m)
    ref = ref_model.forward(W, src, tgt[:, :-1], cfg)
    torch.testing.assert_close(lg.double(), ref.detach(), rtol=1e-4, atol=1e-4)


def test_dropout_is_deterministic_and_scaled():
    cfg = model_config("tiny", d_model=32, heads=4, d_ff=64, src_vocab=50, tgt_vocab=40, dropout=0.1)
    m = Transformer(cfg).build("cpu", seed=4)
    src, tgt = _batch(2, 7, 6, 50, 40, seed=2)
    ctr = torch.zeros(1, dtype=torch.int64)
    rt = RunCtx(training=True, dropout=0.1, seed=9, ctr=ctr, store=None)
    a = m.logits(src, tgt[:, :-1], rt)
    b = m.logits(src, tgt[:, :-1], rt)
    torch.testing.assert_close(a, b)
    ctr += 1
    c = m.logits(src, tgt[:, :-1], rt)
    assert not torch.allclose(a, c)
    e = m.logits(src, tgt[:, :-1], RunCtx(training=False))
    assert not torch.allclose(a, e)


def test_interior_pad_rejected():
    """Keys are masked by length (trailing padding); a PAD before a non-PAD
    token, which the reference would mask position by position
    (transformer_model.py:56-62), is an error rather than a silent mismatch."""
    import pytest
    from tensorflow_distributed_on_gke_amd.models.transformer import seq_lengths

    ok = torch.tensor([[5, 6, 7, 0, 0], [5, 0, 0, 0, 0], [0, 0, 0, 0, 0]])
    assert seq_lengths(ok).tolist() == [3, 1, 0]
    bad = torch.tensor([[5, 0, 7, 0, 0]])
    with pytest.raises(ValueError, match="right-padded"):
        seq_lengths(bad)
