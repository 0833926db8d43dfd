#!/bin/bash
# Fused Q|K|V projection + attention forward: its tests, the per-call lab
# , the headline A/B against ab_old/.
set -uo pipefail
O=gpurun_out/qkvattn
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
echo "== pytest"
timeout -k 10 400 python -u -m pytest -q --maxfail=5 --timeout 200 --timeout-method thread -m gpu tests/test_gpu_qkv_attn.py tests/test_gpu_kernels.py -k "qkv or attn" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -80; exit $rc; }
echo "== lab"
timeout -k 10 200 python -u scripts/qkv_attn_lab.py > $O/lab.log 2>&1 || { tail -20 $O/lab.log; exit 1; }
grep "^B\|^bwd\|^cross" $O/lab.log
[ "${AB:-1}" = "1" ] || exit 0
echo "== pytest model/graph"
timeout -k 10 400 python -u -m pytest -q --maxfail=5 --timeout 200 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_graph.py > $O/pytest2.log 2>&1
rc=$?; tail -2 $O/pytest2.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest2.log | head -80; exit $rc; }
echo "== A/B headline"
bash scripts/ab_trees.sh $PWD/ab_old $PWD ${R:-3} || exit 1
