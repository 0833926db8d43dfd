#!/bin/bash
# persistent fp8 GEMM per epilogue: bitwise test, then config 5 with
# TDG_FP8_PERSIST=0 / default (ReLU fwd + 8-bit-mask ReLU bwd) / all (interleaved)
set -uo pipefail
T=${1:-pk2}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp8.py -k "persistent" \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh $T 3 "TDG_FP8_PERSIST=0" "TDG_FP8_PERSIST=2,4" "TDG_FP8_PERSIST=all" || exit 1
