#!/bin/bash
# e4m3 attention forward ring depth (TDG_ATTN_FWD8_NS 3 / 4 / 6): forward
# tests at each depth, the seq-512 lab at each
set -uo pipefail
T=${1:-fwd8ns}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
for ns in 3 4 6; do
  TDG_ATTN_FWD8_NS=$ns timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fp8.py -k "attention_fwd" \
    > $O/pytest_$ns.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest_$ns.log | head -60; exit 1; }
  tail -1 $O/pytest_$ns.log
  TDG_ATTN_FWD8_NS=$ns ATTN_FP8=1 ATTN_B=16 ATTN_H=16 ATTN_L=512 timeout -k 10 120 python -u scripts/attn_bench.py > $O/lab_$ns.log 2>&1 || { tail -20 $O/lab_$ns.log; exit 1; }
  echo "NS=$ns"; grep "e4m3" $O/lab_$ns.log
done
