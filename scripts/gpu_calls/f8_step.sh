#!/bin/bash
# fp8 step checks: the fp8 / DP GPU tests, then config 5 with and without the
# fp8 attention backward (interleaved)
set -uo pipefail
T=${1:-f8s}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fp8.py tests/test_gpu_attn_f8.py tests/test_gpu_dp.py \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh $T 2 "TDG_ATTN_BWD_F8=0" "TDG_ATTN_BWD_F8=1" || exit 1
grep -h last_loss gpurun_out/ab_$T/v2_1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('loss', d['config']['last_loss'])"
