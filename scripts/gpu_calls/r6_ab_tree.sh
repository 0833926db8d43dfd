#!/bin/bash
# A/B of this tree against the built copy in ab_old/: GPU kernel / model /
# graph tests on this tree, the ragged weight-gradient lab in both, then
# interleaved headline and config-4 benches.
set -uo pipefail
TAG=${1:-r6ab}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
echo "== pytest"
timeout -k 10 600 python -u -m pytest --maxfail=10 -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_graph.py tests/test_gpu_model.py tests/test_gpu_fp8.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -100; exit $rc; }
echo "== wgrad lab (old, new)"
for t in ab_old .; do
  (cd $t && CFGS=12 timeout -k 10 300 python -u scripts/wgrad_lab.py 2>&1 | grep "ragged") | sed "s#^#[$t] #" || exit 1
done
echo "== A/B headline"
bash scripts/ab_trees.sh $PWD/ab_old $PWD 3 || exit 1
