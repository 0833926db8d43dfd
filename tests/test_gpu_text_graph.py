"""Variable-length batches under HIP graphs (the reference's real workload:
every batch padded to its own longest sequence, english_portugese_dataset.py:44-46,
traced with experimental_relax_shapes, __main__.py:127,134).

TrainStep's shape cache (train/step.py, `bucketed`) captures each new batch
shape on first sight -- warm-up steps rolled back, so the batch still trains
once -- and replays the captured step of its shape afterwards, all captures
sharing one memory pool. Checked: a stream of batches of several bucketed
shapes (repeats, a shape returning after others, an eviction from a small
cache) leaves bitwise the weights and losses of the eager step on the same
padded batches; and the training loop with data=text captures and logs its
graph cache."""
import os
import random

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _batches():
    g = torch.Generator().manual_seed(9)
    # (S, T) buckets in a sequence with repeats and returns
    shapes = [(32, 33), (32, 33), (64, 33), (32, 65), (64, 65), (32, 33), (64, 33), (96, 97), (32, 65)]
    out = []
    for i, (S, T) in enumerate(shapes):
        src = torch.randint(4, 500, (8, S), generator=g)
        tgt = torch.randint(4, 400, (8, T), generator=g)
        src[:, S - 7 - i:] = 0  # right padding inside the bucket
        tgt[2:, T - 11 - i:] = 0
        out.append((src.to(DEV), tgt.to(DEV)))
    return out


def _run(bucketed, cache=64, fp8=False):
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    kk.AUTOTUNE = False  # identical GEMM configs in both runs
    cfg = model_config("tiny", d_model=256, heads=4, d_ff=1024, src_vocab=500, tgt_vocab=400, dropout=0.1)
    m = Transformer(cfg).build(DEV, seed=4)
    opt = Adam(m.store, cfg.d_model, lr=0.003)
    st = None
    if fp8:
        from tensorflow_distributed_on_gke_amd.ops.fp8 import Fp8State
        st = Fp8State(m)
    step = TrainStep(m, opt, None, workers=1, seed=6, fp8_state=st)
    bs = _batches()
    if bucketed:
        step.bucketed = True
        step.graph_cache = cache
        assert step.capture(*bs[0])
    losses = [step(*b).clone() for b in bs]
    torch.cuda.synchronize()
    assert opt.iterations == len(bs)
    return m.store.flat.clone(), torch.stack(losses), step


@pytest.mark.parametrize("fp8", [False, True])
def test_bucketed_graph_steps_match_eager(fp8):
    f_e, l_e, _ = _run(False, fp8=fp8)
    f_g, l_g, st = _run(True, fp8=fp8)
    assert st.captured and st.cached_shapes == 5
    assert st.graph_stats["captures"] == 5 and st.graph_stats["evictions"] == 0
    assert torch.equal(l_e, l_g), (l_e, l_g)
    assert torch.equal(f_e, f_g)


def test_bucketed_graph_cache_evicts_lru():
    f_e, l_e, _ = _run(False)
    f_g, l_g, st = _run(True, cache=2)
    assert st.cached_shapes == 2 and st.graph_stats["evictions"] > 0
    assert torch.equal(l_e, l_g)
    assert torch.equal(f_e, f_g)


def test_unbucketed_captured_step_rejects_other_shapes():
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep
    cfg = model_config("tiny", d_model=128, heads=4, d_ff=256, src_vocab=500, tgt_vocab=400)
    m = Transformer(cfg).build(DEV, seed=1)
    step = TrainStep(m, Adam(m.store, cfg.d_model), None, workers=1)
    bs = _batches()
    assert step.capture(*bs[0])
    with pytest.raises(ValueError, match="captured step takes"):
        step(*bs[2])


def test_text_training_loop_captures_buckets(tmp_path):
    """`train --set data=text --set hip_graph=true`: the loop captures per
    length bucket and logs its graph cache."""
    from tensorflow_distributed_on_gke_amd.config import Settings
    from tensorflow_distributed_on_gke_amd.parallel.dist import DistInfo
    from tensorflow_distributed_on_gke_amd.train.loop import Trainer
    rng = random.Random(0)
    words = [f"w{i}" for i in range(300)]
    p = tmp_path / "c.tsv"
    with open(p, "w") as f:
        for _ in range(400):
            n = min(120, int(rng.expovariate(1 / 18)) + 2)
            src = " ".join(rng.choice(words) for _ in range(n))
            tgt = " ".join(rng.choice(words) for _ in range(max(2, n + rng.randint(-3, 3))))
            f.write(f"{src}\t{tgt}\n")
    s = Settings(preset="tiny", data="text", train_file=str(p), src_vocab=400, tgt_vocab=400,
                 local_batch_size=16, epochs=1, log_every=8, snapshot_every_epochs=0, resume=False,
                 hip_graph=True, graph_bucket=32, temporary_directory=str(tmp_path / "tmp"))
    logs = []
    info = DistInfo(rank=0, world=1, local_rank=0, device=torch.device(DEV))
    tr = Trainer(s, info, log=logs.append)
    hist = tr.fit()
    assert tr.step_fn.captured and tr.step_fn.bucketed
    assert 1 < tr.step_fn.cached_shapes <= s.graph_cache
    assert any(line.startswith("graph cache:") for line in logs), logs
    assert hist and hist[0].train_loss == hist[0].train_loss
