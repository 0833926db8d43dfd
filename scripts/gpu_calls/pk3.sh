#!/bin/bash
# persistent fp8 GEMM epilogue set after the write-through stores: default (2,4) vs all
set -uo pipefail
T=${1:-pk3}
export TDG_NO_AUTOBUILD=1
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh $T 3 "TDG_FP8_PERSIST=2,4" "TDG_FP8_PERSIST=all" || exit 1
