#!/bin/bash
# e4m3 attention forward, 16 vs 32 queries per wave: fp8 forward tests, the
# seq-512 timing lab, then config 5 with TDG_ATTN_FWD8_U=1 vs 2 (interleaved)
set -uo pipefail
T=${1:-fwd8u}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp8.py -k "attention" \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
ATTN_FP8=1 ATTN_B=16 ATTN_H=16 ATTN_L=512 timeout -k 10 120 python -u scripts/attn_bench.py > $O/lab.log 2>&1 || { tail -20 $O/lab.log; exit 1; }
grep "B=" $O/lab.log
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh $T 2 "TDG_ATTN_FWD8_U=1" "TDG_ATTN_FWD8_U=2" || exit 1
