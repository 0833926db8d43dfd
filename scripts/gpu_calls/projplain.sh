#!/bin/bash
# fp8 attention-input projections: plain vs write-through output stores
set -uo pipefail
T=${1:-projplain}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fp8.py \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh $T 3 "TDG_FP8_PROJ_PLAIN=0" "TDG_FP8_PROJ_PLAIN=1" || exit 1
