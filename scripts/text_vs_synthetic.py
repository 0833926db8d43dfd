#!/usr/bin/env python3
"""Variable-length (text) training throughput against synthetic full-length
batches of the same mean padded shape, both under HIP graphs, Transformer-base
on one GPU.

The text run uses the reference's pipeline shape (data/text.py: WordPiece
tokenizers trained on the corpus, buffered shuffle, every global batch padded
to its longest pair) on a generated TSV corpus -- random words, sentence
lengths drawn from a long-tailed distribution like TED talk transcripts
(mean ~22 words, tail to ~150) -- with batches padded further to length
buckets (graph_bucket) so the captured-step cache (train/step.py) replays a
graph for most batches. Epoch 1 fills the cache (each new bucket is captured
when it first arrives); epoch 2 is timed. The synthetic run then trains on
full-length batches of the text run's mean padded (source, target) lengths.

    python scripts/text_vs_synthetic.py [--pairs 6400] [--batch 64] [--bucket 32]
Prints one JSON line.
"""
import argparse
import json
import os
import random
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_distributed_on_gke_amd.config import Settings  # noqa: E402
from tensorflow_distributed_on_gke_amd.parallel.dist import DistInfo  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.loop import Trainer  # noqa: E402


def corpus(path, n, seed=0):
    rng = random.Random(seed)
    src_words = [f"p{i}x" for i in range(6000)]
    tgt_words = [f"e{i}y" for i in range(6000)]
    with open(path, "w") as f:
        for _ in range(n):
            k = min(150, max(2, int(rng.lognormvariate(2.9, 0.55))))
            s = " ".join(rng.choice(src_words) for _ in range(k))
            t = " ".join(rng.choice(tgt_words) for _ in range(max(2, k + rng.randint(-4, 4))))
            f.write(f"{s}\t{t}\n")


def run(settings, log):
    info = DistInfo(rank=0, world=1, local_rank=0, device=torch.device("cuda"))
    tr = Trainer(settings, info, log=log)
    hist = tr.fit()
    return tr, hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=6400)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--bucket", type=int, default=32)
    args = ap.parse_args()
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "corpus.tsv")
    corpus(path, args.pairs)
    common = dict(preset="base", local_batch_size=args.batch, snapshot_every_epochs=0, resume=False,
                  hip_graph=True, log_every=10 ** 9, validation_steps=1, temporary_directory=tmp)
    logs = []
    s = Settings(data="text", train_file=path, epochs=2, graph_bucket=args.bucket, **common)
    tr, hist = run(s, logs.append)
    lens = [(tr.train_data.batch(i)[0].shape[1], tr.train_data.batch(i)[1].shape[1])
            for i in range(tr.train_data.steps_per_epoch)]
    mS = sum(a for a, _ in lens) / len(lens)
    mT = sum(b - 1 for _, b in lens) / len(lens)
    text = {"tokens_per_s": round(hist[1].tokens_per_s), "epoch_s": round(hist[1].seconds, 3),
            "steps_per_epoch": tr.train_data.steps_per_epoch, "mean_src_len": round(mS, 1),
            "mean_tgt_in_len": round(mT, 1), "cached_shapes": tr.step_fn.cached_shapes,
            "graph_stats": tr.step_fn.graph_stats,
            "vocab": [tr.model.cfg.src_vocab, tr.model.cfg.tgt_vocab]}
    del tr
    torch.cuda.empty_cache()
    S, T = int(round(mS)), int(round(mT))
    s2 = Settings(data="synthetic", src_len=S, tgt_len=T, src_vocab=text["vocab"][0],
                  tgt_vocab=text["vocab"][1], epochs=2, steps_per_epoch=text["steps_per_epoch"],
                  min_len=4, **common)
    _, h2 = run(s2, lambda m: None)
    syn = {"tokens_per_s": round(h2[1].tokens_per_s), "src_len": S, "tgt_in_len": T}
    print(json.dumps({"text": text, "synthetic_matched": syn,
                      "text_over_synthetic": round(text["tokens_per_s"] / syn["tokens_per_s"], 3)}),
          flush=True)


if __name__ == "__main__":
    main()
