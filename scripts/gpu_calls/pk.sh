#!/bin/bash
# persistent fp8 GEMM: bitwise test vs the one-shot grid, the K sweep with it
# on / off, then config 5 with TDG_FP8_PERSIST=0 / 1 (interleaved)
set -uo pipefail
T=${1:-pk}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp8.py -k "persistent or gemm" \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
for p in 0 1; do
  TDG_FP8_PERSIST=$p timeout -k 10 300 python -u scripts/fp8_ksweep.py > $O/ksweep_$p.log 2>&1 || { tail -20 $O/ksweep_$p.log; exit 1; }
  echo "persist=$p"; grep -v amdgpu.ids $O/ksweep_$p.log
done
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh $T 2 "TDG_FP8_PERSIST=0" "TDG_FP8_PERSIST=1" || exit 1
