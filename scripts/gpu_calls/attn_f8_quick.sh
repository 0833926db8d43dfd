#!/bin/bash
# fp8 attention backward: numerics + lab timing (+ PMC of the lab)
set -uo pipefail
T=${1:-af8q}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_attn_f8.py \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u scripts/attn_f8_lab.py > $O/lab.txt 2>&1 || { tail -20 $O/lab.txt; exit 1; }
grep causal $O/lab.txt
[ "${PMC:-1}" = "1" ] && bash scripts/gpu_calls/attn_f8_pmc.sh $T/pmc | grep -A16 "attn_bwd_f8"
exit 0
