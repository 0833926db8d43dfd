#!/bin/bash
# e5m2 cross K|V gradient from the fp8 attention backward: fp8 tests, then
# config 5 against the previous build (ab_old/)
set -uo pipefail
T=${1:-kv8}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fp8.py tests/test_gpu_attn_f8.py \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for t in ab_old .; do
    n=$(basename $(cd $t && pwd))
    (cd $t && timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 > /tmp/b_$n.log 2>&1) || { echo "$t failed"; tail -5 /tmp/b_$n.log; exit 1; }
    echo "[$n] run=$r $(tail -1 /tmp/b_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["last_loss"])')"
  done
done
