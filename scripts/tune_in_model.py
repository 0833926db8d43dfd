#!/usr/bin/env python3
"""In-situ GEMM tile selection: time whole eager training steps while one
GEMM shape's tile config is varied, all others held at the current table.

The isolated autotuner (ops/kernels.py) times a GEMM back-to-back with warm
caches; inside the step, epilogue operands (the ReLU mask written in forward,
the residual gradient) and weights are cold and neighbouring kernels contend
for L2/MALL, so the best isolated tile is not always the best in the step.
Each candidate is measured in interleaved rounds (median of rounds), and the
winning table is written as JSON (same format as gemm_tuned_gfx950.json).

    python scripts/tune_in_model.py --preset base --out gpurun_out/tuned_inmodel.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs  # noqa: E402
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config  # noqa: E402
from tensorflow_distributed_on_gke_amd.ops import kernels as kk  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.optim import Adam  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.step import TrainStep  # noqa: E402

CANDS = [(c, 1) for c in (0, 4, 5, 6, 9, 10, 12, 13, 14, 20, 21, 22)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="base")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--min-flops", type=float, default=2e9)
    ap.add_argument("--out", default="gpurun_out/tuned_inmodel.json")
    ap.add_argument("--epi", type=lambda v: [int(x) for x in v.split(",")], default=None,
                    help="only GEMMs with these epilogues (e.g. 1,2: bias, bias+relu)")
    ap.add_argument("--graph", type=int, default=0,
                    help="time HIP-graph replays (one capture per candidate) instead of eager steps")
    ap.add_argument("--cands", type=lambda v: [(int(x), 1) for x in v.split(",")], default=None,
                    help="tile configs to try (default: CANDS)")
    args = ap.parse_args()

    dev = torch.device("cuda", 0)
    cfg = model_config(args.preset)
    model = Transformer(cfg).build(dev, seed=0)
    opt = Adam(model.store, cfg.d_model)
    step = TrainStep(model, opt, None, workers=1.0, seed=17)
    data = SyntheticPairs(batch=args.batch, src_len=args.seq_len, tgt_len=args.seq_len + 1,
                          src_vocab=cfg.src_vocab, tgt_vocab=cfg.tgt_vocab, seed=0)
    s, t = data.batch(0)
    s, t = s.to(dev), t.to(dev)

    # record the GEMM keys one step uses (and whether the library path applies)
    seen = {}
    orig = kk.gemm

    def spy(A, B, Cout, M, N, K, lda, ldb, ldc, a_kc, b_kc, epi=kk.EPI_NONE, bias=None, aux=None,
            ldaux=0, alpha=1.0, beta=0.0, cfg=None):
        Mk, Kk = (M, kk._tok_bucket(K)) if (not a_kc and not b_kc) else (kk._tok_bucket(M), K)
        key = (Mk, N, Kk, a_kc, b_kc, epi, Cout.dtype, ldc % 8 == 0, beta != 0.0)
        if cfg is None and (not args.epi or epi in args.epi):
            seen.setdefault(key, [0, False])[0] += 1
        return orig(A, B, Cout, M, N, K, lda, ldb, ldc, a_kc, b_kc, epi, bias, aux, ldaux, alpha, beta,
                    cfg)

    kk.gemm = spy
    for _ in range(3):
        step(s, t)
    torch.cuda.synchronize()
    kk.gemm = orig

    def timed():
        if args.graph:
            step.capture(s, t)  # (the current table, captured)
        for _ in range(3):
            step(s, t)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.steps):
            step(s, t)
        b.record()
        b.synchronize()
        return a.elapsed_time(b) / args.steps * 1e3  # us per step

    base = timed()
    print(f"start: {base:.1f} us/step, {len(seen)} GEMM shapes", flush=True)
    for key, (calls, blas_ok) in sorted(seen.items(), key=lambda kv: -kv[0][0] * kv[0][1] * kv[0][2] * kv[1][0]):
        M, N, K = key[:3]
        if 2.0 * M * N * K * calls < args.min_flops:
            continue
        cur = kk._TUNED.get(key, (None,))[0]
        cands = list(args.cands or CANDS)
        if cur is not None and cur not in cands:
            cands.append(cur)
        times = {c: [] for c in cands}
        for _ in range(args.rounds):
            for c in cands:
                kk._TUNED[key] = (c, c)
                try:
                    times[c].append(timed())
                except RuntimeError:
                    times[c].append(float("inf"))
        med = {c: sorted(v)[len(v) // 2] for c, v in times.items()}
        best = min(med, key=med.get)
        kk._TUNED[key] = (best, best)
        print(json.dumps({"key": kk._key_str(key), "calls": calls, "was": cur, "best": best,
                          "us_step": {f"{c[0]}": round(v, 1) for c, v in med.items()}}), flush=True)
    final = timed()
    print(f"end: {final:.1f} us/step (start {base:.1f})", flush=True)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    kk.save_tuned(args.out)


if __name__ == "__main__":
    main()
