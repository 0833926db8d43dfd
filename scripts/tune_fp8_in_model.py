#!/usr/bin/env python3
"""In-model tile selection for the fp8 forward GEMMs (ops/fp8.py gemm_fp8):
the shapes one eager fp8 training step runs are collected, then for each
shape (largest first) every candidate tile config is timed over whole eager
steps with all other shapes held at the current choice (interleaved rounds,
median), and the winners are written as the fp8 tuned table (JSON,
ops/fp8_tuned_gfx950.json format).

    python scripts/tune_fp8_in_model.py --out gpurun_out/fp8_tuned.json
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs  # noqa: E402
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config  # noqa: E402
from tensorflow_distributed_on_gke_amd.ops import fp8 as F  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.optim import Adam  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.step import TrainStep  # noqa: E402

CANDS = (0, 1, 2, 3, 4, 5, 8, 9, 10)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="big")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--seq-len", type=int, default=512)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/fp8_tuned.json")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = model_config(args.preset, max_src_len=max(1000, args.seq_len), max_tgt_len=max(1000, args.seq_len))
    model = Transformer(cfg).build(dev, seed=0)
    opt = Adam(model.store, cfg.d_model)
    st = F.Fp8State(model)
    step = TrainStep(model, opt, None, workers=1.0, seed=17, fp8_state=st)
    data = SyntheticPairs(batch=args.batch, src_len=args.seq_len, tgt_len=args.seq_len + 1,
                          src_vocab=cfg.src_vocab, tgt_vocab=cfg.tgt_vocab, seed=0)
    batch = [t.to(dev) for t in data.batch(0)]
    F._TUNED.clear()
    step(*batch)  # every fp8 forward shape gets its default choice
    torch.cuda.synchronize()
    keys = sorted(F._TUNED, key=lambda k: -k[0] * k[1] * k[2])
    print("shapes:", keys, flush=True)

    def run_steps():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(*batch)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3

    for _ in range(2):
        run_steps()
    for key in keys:
        best = {}
        for r in range(args.rounds):
            for c in CANDS:
                F._TUNED[key] = c
                try:
                    t = run_steps()
                except RuntimeError as e:  # unsupported config for this shape
                    print(f"  {key} cfg {c}: {e}".splitlines()[0], flush=True)
                    torch.cuda.synchronize()
                    continue
                best.setdefault(c, []).append(t)
        med = {c: sorted(v)[len(v) // 2] for c, v in best.items() if len(v) == args.rounds}
        win = min(med, key=med.get)
        F._TUNED[key] = win
        print(f"{key}: " + "  ".join(f"c{c}={t:.3f}" for c, t in sorted(med.items())) + f"  -> {win}",
              flush=True)
    F.save_tuned(args.out)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
