#!/bin/bash
# in-model fp8 forward tile selection for config 5, then an A/B of the table
set -uo pipefail
T=${1:-f8tune}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 900 python -u scripts/tune_fp8_in_model.py --out $O/fp8_tuned.json > $O/tune.log 2>&1 || { tail -30 $O/tune.log; exit 1; }
cat $O/tune.log | grep -v amdgpu.ids
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh $T 2 "-" "TDG_FP8_TUNED_FILE=$O/fp8_tuned.json" || exit 1
