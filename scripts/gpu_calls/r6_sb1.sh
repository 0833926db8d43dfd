#!/bin/bash
# Fused self-attention forward, single-buffered 2-workgroup-per-CU variant
# (TDG_QKV_ATTN_SB1=1) against the default: tests, lab, headline A/B.
set -uo pipefail
O=gpurun_out/sb1
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
echo "== pytest (SB1)"
TDG_QKV_ATTN_SB1=1 timeout -k 10 300 python -u -m pytest -q --maxfail=5 --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -80; exit $rc; }
echo "== lab"
for v in 0 1; do
  TDG_QKV_ATTN_SB1=$v timeout -k 10 200 python -u scripts/qkv_attn_lab.py > $O/lab_$v.log 2>&1 || { tail -20 $O/lab_$v.log; exit 1; }
  grep "^B" $O/lab_$v.log | sed "s/^/[SB1=$v] /"
done
echo "== A/B"
bash scripts/ab_env.sh sb1 3 "TDG_QKV_ATTN_SB1=0" "TDG_QKV_ATTN_SB1=1"
