#!/bin/bash
# XCD-grouped attention workgroup order: attention tests, then headline and
# config-5 A/B (TDG_ATTN_XCD=0 plain grid order vs 1)
set -uo pipefail
T=${1:-axcd}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_attn_f8.py -k "attn or attention" \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
bash scripts/ab_env.sh ${T}_base 3 "TDG_ATTN_XCD=0" "TDG_ATTN_XCD=1" || exit 1
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh ${T}_f8 2 "TDG_ATTN_XCD=0" "TDG_ATTN_XCD=1" || exit 1
