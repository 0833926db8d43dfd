"""Real-text data path (data/text.py): WordPiece tokenizers with the reference
converter's reserved ids, the tf.data-style pipeline (cache, buffered shuffle
re-drawn per epoch, global batches, DATA sharding, pad to the global batch's
longest sequence) and a 2-rank CPU training run on a generated pt/en corpus.
The reference's TED corpus and SavedModel converter are not available (no
network, no TensorFlow): tokenisation parity with them is unpinned."""
import os
import random
import subprocess
import sys

import pytest
import torch

from tensorflow_distributed_on_gke_amd.data.text import (END, PAD, START, TextPairs, WordPieceTokenizer,
                                                        buffered_shuffle, read_pairs)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PT = {"gato": "cat", "cão": "dog", "casa": "house", "livro": "book", "carro": "car",
       "menina": "girl", "menino": "boy", "água": "water", "escola": "school", "cidade": "city"}
_ADJ = {"grande": "big", "pequeno": "small", "novo": "new", "velho": "old", "bonito": "beautiful"}


def _corpus(path, n=240, seed=0):
    rng = random.Random(seed)
    nouns, adjs = list(_PT), list(_ADJ)
    with open(path, "w", encoding="utf-8") as f:
        for i in range(n):
            k = rng.randint(1, 3)
            ps, es = [], []
            for _ in range(k):
                a, b = rng.choice(nouns), rng.choice(adjs)
                ps.append(f"o {a} é {b}")
                es.append(f"the {_PT[a]} is {_ADJ[b]}")
            f.write(" e ".join(ps) + " .\t" + " and ".join(es) + " .\n")
        f.write("linha sem tabulação\n\n")  # skipped
    return path


def test_wordpiece_reserved_ids_roundtrip_and_save(tmp_path):
    p = _corpus(tmp_path / "c.tsv")
    pairs = read_pairs(str(p))
    assert len(pairs) == 240
    tok = WordPieceTokenizer.train((s for s, _ in pairs), vocab_size=200)
    assert [tok.lookup([i])[0] for i in range(4)] == ["[PAD]", "[UNK]", "[START]", "[END]"]
    ids = tok.encode("o gato é grande")
    assert ids[0] == START and ids[-1] == END and all(i > END for i in ids[1:-1])
    assert tok.detokenize(ids) == "o gato e grande" or tok.detokenize(ids) == "o gato é grande"
    t = tok.tokenize(["o gato", "o cão é pequeno e velho"])
    assert t.dtype == torch.int64 and t[0, -1] == PAD and t[1, -1] != PAD
    tok.save(str(tmp_path / "t.json"))
    tok2 = WordPieceTokenizer.load(str(tmp_path / "t.json"))
    assert tok2.encode("a escola nova") == tok.encode("a escola nova")
    assert tok2.vocab_size == tok.vocab_size <= 200


def test_buffered_shuffle_is_a_seeded_permutation():
    for n, buf in ((100, 7), (100, 1000), (50, 1)):
        o = buffered_shuffle(n, buf, seed=3)
        assert sorted(o) == list(range(n))
        assert o == buffered_shuffle(n, buf, seed=3)
    assert buffered_shuffle(50, 1, 0) == list(range(50))  # buffer 1: no shuffle
    # tf.data semantics: an element cannot be emitted before it entered the buffer
    o = buffered_shuffle(1000, 10, seed=1)
    assert all(idx < pos + 10 for pos, idx in enumerate(o))


def test_text_pairs_sharding_padding_epochs(tmp_path):
    p = str(_corpus(tmp_path / "c.tsv"))
    pairs = read_pairs(p)
    st = WordPieceTokenizer.train((s for s, _ in pairs), 200)
    tt = WordPieceTokenizer.train((t for _, t in pairs), 150)
    world, lb = 3, 8
    ranks = [TextPairs(p, st, tt, lb, r, world, seed=5, shuffle_buffer=64) for r in range(world)]
    assert ranks[0].steps_per_epoch == 240 // 24
    for step in (0, 3, 11):  # 11 wraps into epoch 2
        parts = [r.batch(step) for r in ranks]
        # one global batch: identical padded lengths on every rank
        assert len({s.shape[1] for s, _ in parts}) == 1 and len({t.shape[1] for _, t in parts}) == 1
        src = torch.cat([s for s, _ in parts])
        tgt = torch.cat([t for _, t in parts])
        assert src.shape[0] == world * lb
        # padded to the longest row of the global batch; every row [START] .. [END] then PAD
        assert ((src != PAD).sum(1).max() == src.shape[1]) and ((tgt != PAD).sum(1).max() == tgt.shape[1])
        for row in tgt:
            n = int((row != PAD).sum())
            assert row[0] == START and row[n - 1] == END and (row[n:] == PAD).all()
    # disjoint rank slices cover each global batch; an epoch covers the data once
    seen = []
    for step in range(ranks[0].steps_per_epoch):
        for r in ranks:
            s, _ = r.batch(step)
            seen += [tuple(x[x != PAD].tolist()) for x in s]
    want = sorted(tuple(st.encode(a)) for a, _ in pairs)
    assert sorted(seen) == want
    # reshuffled every epoch, deterministic per seed
    e0 = [r.batch(0)[0] for r in ranks]
    e1 = [r.batch(ranks[0].steps_per_epoch)[0] for r in ranks]
    assert any(a.shape != b.shape or not torch.equal(a, b) for a, b in zip(e0, e1))
    again = TextPairs(p, st, tt, lb, 1, world, seed=5, shuffle_buffer=64)
    assert torch.equal(again.batch(4)[0], ranks[1].batch(4)[0])
    # next / seek follow batch()
    again.seek(7)
    assert torch.equal(again.next()[1], ranks[1].batch(7)[1])
    with pytest.raises(ValueError):
        TextPairs(p, st, tt, 100, 0, 3)


def test_train_cli_on_text_data_two_ranks(tmp_path):
    """`train` with data=text on 2 gloo ranks: tokenizers trained from the
    corpus and saved, the model sized by their vocabularies, loss falls, and
    `test` translates with the saved tokenizers."""
    _corpus(tmp_path / "train.tsv", n=256, seed=1)
    _corpus(tmp_path / "val.tsv", n=64, seed=2)
    port = 29000 + os.getpid() % 2000
    cmd = [sys.executable, "-m", "tensorflow_distributed_on_gke_amd", "train", "--nproc", "2",
           "--master-port", str(port), "--config", os.path.join(ROOT, "configuration", "settings.yaml")]
    sets = ["data=text", "train_file=train.tsv", "validation_file=val.tsv", "preset=tiny",
            "local_batch_size=16", "src_vocab=120", "tgt_vocab=100", "epochs=4", "log_every=4",
            "snapshot_every_epochs=0", "learning_rate=0.003", "worker_count=2", "dropout=0.0",
            "resume=false"]
    for kv in sets:
        cmd += ["--set", kv]
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("RANK", None)
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    losses = [float(line.split("Loss ")[1].split()[0]) for line in r.stdout.splitlines()
              if line.startswith("Epoch ") and " Batch " not in line and "Loss" in line]
    assert len(losses) == 4 and losses[-1] < 0.8 * losses[0], r.stdout
    assert (tmp_path / "temporary" / "tokenizer_src.json").exists()
    t = subprocess.run([sys.executable, "-m", "tensorflow_distributed_on_gke_amd", "test", "--device", "cpu",
                        "--config", os.path.join(ROOT, "configuration", "settings.yaml"),
                        "--set", "preset=tiny", "--set", "src_tokenizer=temporary/tokenizer_src.json",
                        "--set", "tgt_tokenizer=temporary/tokenizer_tgt.json",
                        "--sentence", "o gato é grande ."],
                       cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert t.returncode == 0, t.stdout + t.stderr
    assert "'o gato é grande .' ->" in t.stdout and "attention maps" in t.stdout


def test_bucketed_batches_pad_to_length_buckets(tmp_path):
    """bucket > 1 (hip_graph text runs): every batch is padded further, the
    source to a multiple of the bucket and the target so that the decoder
    input (target minus the shifted token) is one, never past max_len, and
    the extra columns are PAD only (the rows are the unbucketed ones)."""
    from tensorflow_distributed_on_gke_amd.data.text import bucket_lengths
    assert bucket_lengths(5, 9, 1, 1000) == (5, 9)
    assert bucket_lengths(5, 9, 32, 1000) == (32, 33)
    assert bucket_lengths(32, 33, 32, 1000) == (32, 33)
    assert bucket_lengths(33, 34, 32, 1000) == (64, 65)
    assert bucket_lengths(990, 1000, 32, 1000) == (992, 1000)  # capped at max_len
    assert bucket_lengths(999, 990, 32, 1000) == (1000, 993)
    p = _corpus(tmp_path / "c.tsv")
    tok_s = WordPieceTokenizer.train((s for s, _ in read_pairs(str(p))), vocab_size=200)
    tok_t = WordPieceTokenizer.train((t for _, t in read_pairs(str(p))), vocab_size=200)
    plain = TextPairs(str(p), tok_s, tok_t, local_batch=8, seed=1)
    bk = TextPairs(str(p), tok_s, tok_t, local_batch=8, seed=1, bucket=16)
    shapes = set()
    for i in range(plain.steps_per_epoch):
        (s0, t0), (s1, t1) = plain.batch(i), bk.batch(i)
        assert s1.shape[1] % 16 == 0 and (t1.shape[1] - 1) % 16 == 0
        assert torch.equal(s1[:, :s0.shape[1]], s0) and bool((s1[:, s0.shape[1]:] == PAD).all())
        assert torch.equal(t1[:, :t0.shape[1]], t0) and bool((t1[:, t0.shape[1]:] == PAD).all())
        shapes.add((tuple(s1.shape), tuple(t1.shape)))
    assert len(shapes) < plain.steps_per_epoch
