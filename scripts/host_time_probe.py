"""Host-side cost of one eager training step (Transformer-base, batch 64 x 128):
wall time of the Python/launch work with the GPU kept busy, vs the GPU time.
If host time >= GPU time the eager (data-parallel) step is launch-bound."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
from tensorflow_distributed_on_gke_amd.train.optim import Adam
from tensorflow_distributed_on_gke_amd.train.step import TrainStep


def main():
    m = Transformer(model_config("base", dropout=0.1)).build("cuda", seed=0)
    opt = Adam(m.store, m.cfg.d_model)
    step = TrainStep(m, opt, None, workers=1, seed=1)
    data = SyntheticPairs(64, 128, 129, m.cfg.src_vocab, m.cfg.tgt_vocab, seed=0)
    src, tgt = (t.cuda() for t in data.batch(0))
    for _ in range(10):
        step(src, tgt)
    torch.cuda.synchronize()
    n = 30
    t0 = time.perf_counter()
    for _ in range(n):
        step(src, tgt)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"back-to-back: host {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step")
    # one step from an idle GPU: the host's enqueue cost vs the step's GPU time
    hs, ws = [], []
    for _ in range(15):
        torch.cuda.synchronize()
        a = time.perf_counter()
        step(src, tgt)
        b = time.perf_counter()
        torch.cuda.synchronize()
        c = time.perf_counter()
        hs.append(b - a)
        ws.append(c - a)
    hs.sort()
    ws.sort()
    print(f"single step from idle: host enqueue {1e3 * hs[7]:.3f} ms, wall {1e3 * ws[7]:.3f} ms (medians)")
    import cProfile
    import pstats
    pr = cProfile.Profile()
    for _ in range(10):  # profile the enqueue of single steps from an idle GPU (no blocking)
        torch.cuda.synchronize()
        pr.enable()
        step(src, tgt)
        pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(45)


if __name__ == "__main__":
    main()
