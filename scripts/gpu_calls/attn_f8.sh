#!/bin/bash
# fp8 attention backward: numerics tests, the fp8 model tests, then a
# config-5 A/B (fp8 attention backward on / off) and its kernel trace.
set -uo pipefail
T=${1:-af8}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_attn_f8.py \
  > $O/pytest_f8.log 2>&1 || { tail -40 $O/pytest_f8.log; exit 1; }
grep -E "PASS|FAIL" $O/pytest_f8.log | tail -12
timeout -k 10 120 python -u scripts/attn_f8_lab.py > $O/lab.txt 2>&1 || { tail -20 $O/lab.txt; exit 1; }
cat $O/lab.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fp8.py tests/test_gpu_dp.py \
  > $O/pytest_fp8.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest_fp8.log | head -60; exit 1; }
tail -2 $O/pytest_fp8.log
BENCH_ARGS="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5" \
  bash scripts/ab_env.sh f8bwd 2 "TDG_ATTN_BWD_F8=0" "TDG_ATTN_BWD_F8=1" || exit 1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p8 -o p -- python3 bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 10 --warmup 3 --graph 0 > $O/p8.log 2>&1 || { tail -20 $O/p8.log; exit 1; }
f=$(find $O/p8 -name "*kernel_stats.csv" | head -1)
python3 scripts/kstats.py "$f" 13 > $O/p8.txt
head -24 $O/p8.txt
