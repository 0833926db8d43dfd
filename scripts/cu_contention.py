#!/usr/bin/env python3
"""How sensitive is the training step to losing CUs to a concurrent kernel?

At N > 1 the RCCL all-reduce workgroups occupy CUs while backward runs; most
of our GEMMs launch exactly one tile per CU, so a few missing CUs can push a
launch into a second round of tiles. This runs the single-GPU HIP-graph step
(Transformer-base, batch 64 x 128) alone and with a memory-streaming kernel
of `nblocks` workgroups (ops: cu_hog) on a second stream, launched right
before each replay and sized to last ~2 ms alone: "stream" workgroups read
1 MiB slices in a loop (bandwidth + occupancy), "sleep" workgroups only hold
their CUs (s_sleep). Reports ms/step and the hog's own duration.

    python scripts/cu_contention.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs  # noqa: E402
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config  # noqa: E402
from tensorflow_distributed_on_gke_amd.ops._ext import C  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.optim import Adam  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.step import TrainStep  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg = model_config("base")
    model = Transformer(cfg).build(dev, seed=0)
    opt = Adam(model.store, cfg.d_model)
    step = TrainStep(model, opt, None, workers=1.0, seed=17)
    data = SyntheticPairs(batch=64, src_len=128, tgt_len=129, src_vocab=cfg.src_vocab,
                          tgt_vocab=cfg.tgt_vocab, seed=0)
    s, t = data.batch(0)
    s, t = s.to(dev), t.to(dev)
    step.capture(s, t)
    for _ in range(5):
        step(s, t)
    side = torch.cuda.Stream()
    buf = torch.rand(256 << 18, device=dev)  # 256 MiB
    out = torch.zeros(256, device=dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def hog_alone(nb, iters):
        ev[0].record()
        C().cu_hog(buf, out, nb, iters)
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1])

    def steps(n, nb=0, iters=0):
        torch.cuda.synchronize()
        ev[0].record()
        for _ in range(n):
            if nb:
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    C().cu_hog(buf, out, nb, iters)
            step(s, t)
        ev[1].record()
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / n

    def size(nb, sign):
        # iterations for ~2 ms alone (negative: sleep-only occupancy)
        it = 64 * sign
        hog_alone(nb, it)
        t1 = hog_alone(nb, it)
        return int(it * 2.0 / max(t1, 1e-3))

    res = {"alone_ms": round(steps(30), 3)}
    for kind, sign in (("stream", 1), ("sleep", -1)):
        for nb in (8, 32, 64):
            it = size(nb, sign)
            th = hog_alone(nb, it)
            res[f"{kind}{nb}"] = {"hog_alone_ms": round(th, 3), "step_ms": round(steps(30, nb, it), 3)}
            print(json.dumps(res), flush=True)
    res["alone_ms_again"] = round(steps(30), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
