#!/usr/bin/env python3
"""Timing probe: does running the batch as two concurrent half-batch chains
on two HIP streams (one graph) beat the single full-batch chain?

Not a training path -- the two halves' weight-gradient launches both write
the gradient buffer (timing only). Prints ms per replay for
  single : loss_and_backward(B) + Adam
  seq2   : two half batches one after the other on one stream + Adam
  conc2  : the two half batches on two streams (fork/join) + Adam
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.optim import Adam  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.step import TrainStep  # noqa: E402
from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs  # noqa: E402


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "base"
    B, L = 64, 128
    dev = torch.device("cuda:0")
    cfg = model_config(preset)
    model = Transformer(cfg).build(dev, seed=0)
    opt = Adam(model.store, cfg.d_model)
    step = TrainStep(model, opt, None, workers=1, seed=17)
    data = SyntheticPairs(batch=B, src_len=L, tgt_len=L + 1, src_vocab=cfg.src_vocab,
                          tgt_vocab=cfg.tgt_vocab, seed=0, rank=0, world=1, pin=True)
    s, t = data.batch(0)
    src, tgt = s.to(dev), t.to(dev)
    rt = step.rt
    h = B // 2
    halves = [(src[:h].contiguous(), tgt[:h].contiguous()), (src[h:].contiguous(), tgt[h:].contiguous())]

    def lb(a, b):
        model.loss_and_backward(a, b, rt, 1.0, accum=step.accum, step_out=step.last, bump_ctr=True)

    def single():
        lb(src, tgt)
        opt.apply()

    def seq2():
        for a, b in halves:
            lb(a, b)
        opt.apply()

    sB = torch.cuda.Stream()

    def conc2():
        cur = torch.cuda.current_stream()
        sB.wait_stream(cur)
        lb(*halves[0])
        with torch.cuda.stream(sB):
            lb(*halves[1])
        cur.wait_stream(sB)
        opt.apply()

    graphs = {}
    for name, fn in (("single", single), ("seq2", seq2), ("conc2", conc2)):
        cs = torch.cuda.Stream()
        cs.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cs):
            for _ in range(2):
                fn()
        torch.cuda.current_stream().wait_stream(cs)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        graphs[name] = g
        torch.cuda.synchronize()
    res = {k: [] for k in graphs}
    for rnd in range(4):
        for name, g in graphs.items():
            for _ in range(3):
                g.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                g.replay()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / 20 * 1e3)
    for name, v in res.items():
        print(f"{preset} {name:7s} ms/step min {min(v):.3f} all {[round(x, 3) for x in v]}", flush=True)


if __name__ == "__main__":
    main()
