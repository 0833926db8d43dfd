#!/usr/bin/env python3
"""Host cost of the segmented data-parallel step on one rank (--force-dp
path): back-to-back host vs wall time per step, and the host time of every
replay item (graph launches and recorded collective calls)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29611")
os.environ.setdefault("RANK", "0")
os.environ.setdefault("WORLD_SIZE", "1")
os.environ.setdefault("LOCAL_RANK", "0")

import torch  # noqa: E402

from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs  # noqa: E402
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config  # noqa: E402
from tensorflow_distributed_on_gke_amd.parallel import dist as tdist  # noqa: E402
from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.optim import Adam  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.step import TrainStep  # noqa: E402


def main():
    info = tdist.init_distributed(force=True)
    m = Transformer(model_config("base")).build(info.device, seed=0)
    opt = Adam(m.store, m.cfg.d_model)
    ddp = DataParallel(m.store, bucket_mb=64.0, force=True)
    ddp.broadcast_params(0)
    step = TrainStep(m, opt, ddp, workers=1, seed=1)
    data = SyntheticPairs(64, 128, 129, m.cfg.src_vocab, m.cfg.tgt_vocab, seed=0)
    src, tgt = (t.cuda() for t in data.batch(0))
    ok = step.capture(src, tgt)
    print(f"captured: {ok} mode={step.capture_mode()}")
    for _ in range(10):
        step(src, tgt)
    torch.cuda.synchronize()
    n = 40
    t0 = time.perf_counter()
    for _ in range(n):
        step(src, tgt)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"back-to-back: host {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step")
    seg = step.segments
    if seg is not None:
        print(f"{seg.num_graphs} graphs, {seg.num_calls} host calls per step")
        # per-item host time, GPU kept busy by the preceding steps
        times = [0.0] * len(seg.items)
        reps = 20
        for _ in range(reps):
            for i, (kind, x) in enumerate(seg.items):
                a = time.perf_counter()
                x.replay() if kind == "graph" else x()
                times[i] += time.perf_counter() - a
        torch.cuda.synchronize()
        for i, (kind, _) in enumerate(seg.items):
            print(f"  item {i:2d} {kind:5s} {1e6 * times[i] / reps:8.1f} us")
        print(f"  total {1e3 * sum(times) / reps:.3f} ms")
    tdist.shutdown()


if __name__ == "__main__":
    main()
