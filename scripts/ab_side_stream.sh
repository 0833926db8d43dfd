#!/bin/bash
# Tune once (saved table), then interleave bench runs with / without the side stream.
set -euo pipefail
mkdir -p gpurun_out
TDG_GEMM_TUNED=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --save-tuned gpurun_out/gemm_tuned.json > gpurun_out/ab_tune.log 2>&1
cp gpurun_out/gemm_tuned.json tensorflow_distributed_on_gke_amd/ops/gemm_tuned_gfx950.json
for i in 1 2; do
  for ss in 0 1; do
    TDG_SIDE_STREAM=$ss timeout -k 10 200 python bench.py --steps 40 --warmup 10 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('side=$ss', d['ms_per_step'])"
  done
done
