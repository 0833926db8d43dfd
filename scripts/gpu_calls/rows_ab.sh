#!/bin/bash
# Row reductions on v_permlane16/32_swap (softmax row max, LSE / delta sums):
# attention tests, the e4m3 forward lab, then interleaved A/Bs against the
# previous build (ab_old/): headline bench, then config 5
set -uo pipefail
T=${1:-rows}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_fp8.py tests/test_gpu_attn_f8.py -k "attn or attention" \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
ATTN_FP8=1 ATTN_B=16 ATTN_H=16 ATTN_L=512 timeout -k 10 120 python -u scripts/attn_bench.py > $O/lab512.log 2>&1 || { tail -20 $O/lab512.log; exit 1; }
grep "B=" $O/lab512.log
timeout -k 10 120 python -u scripts/attn_bench.py > $O/lab128.log 2>&1 || { tail -20 $O/lab128.log; exit 1; }
grep "B=" $O/lab128.log
bash scripts/ab_trees.sh ab_old . 3 || exit 1
for r in 1 2; do
  for t in ab_old .; do
    n=$(basename $(realpath $t))
    (cd $t && timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 > $OLDPWD/$O/f8_${n}_$r.log 2>&1) || { echo "$t fp8 failed"; exit 1; }
    echo "[fp8 $n] run=$r $(tail -1 $O/f8_${n}_$r.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step"
  done
done
