#!/usr/bin/env python3
"""Probe: do two half-batch training steps on two streams (two model
replicas, each its own captured HIP graph) finish faster than one full-batch
step? Tests whether cross-stream kernel interleaving fills the latency-bound
gaps (kernel boundaries, prologue / epilogue tails) of the Transformer-base
step. Prints ms per 64-sequence step for each arrangement."""
import os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
from tensorflow_distributed_on_gke_amd.train.optim import Adam
from tensorflow_distributed_on_gke_amd.train.step import TrainStep
from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs

dev = torch.device("cuda", 0)
cfg = model_config("base")


def make(batch, seed):
    m = Transformer(cfg).build(dev, seed=seed)
    st = TrainStep(m, Adam(m.store, cfg.d_model), None, workers=1.0, seed=seed + 17)
    d = SyntheticPairs(batch=batch, src_len=128, tgt_len=129, src_vocab=cfg.src_vocab,
                       tgt_vocab=cfg.tgt_vocab, seed=seed)
    s, t = d.batch(0)
    s, t = s.to(dev), t.to(dev)
    assert st.capture(s, t)
    return st, s, t


full = make(64, 0)
a = make(32, 1)
b = make(32, 2)
sa, sb = torch.cuda.Stream(), torch.cuda.Stream()


def run_full(n):
    for _ in range(n):
        full[0](full[1], full[2])


def run_pair(n):
    for _ in range(n):
        with torch.cuda.stream(sa):
            a[0](a[1], a[2])
        with torch.cuda.stream(sb):
            b[0](b[1], b[2])
    torch.cuda.current_stream().wait_stream(sa)
    torch.cuda.current_stream().wait_stream(sb)


def run_serial_halves(n):
    for _ in range(n):
        a[0](a[1], a[2])
        b[0](b[1], b[2])


def timed(fn, n=30, rounds=5):
    fn(3)
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(n)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) / n * 1e3)
    return sorted(ts)[len(ts) // 2]


for r in range(2):
    print(f"round {r}: full b64 {timed(run_full):.3f} ms | two b32 streams {timed(run_pair):.3f} ms | "
          f"two b32 serial {timed(run_serial_halves):.3f} ms", flush=True)
