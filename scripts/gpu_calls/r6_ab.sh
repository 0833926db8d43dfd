#!/bin/bash
# A/B session: GPU tests (a selection), the headline interleaved against the
# built copy of the previous commit in ab_old/, then a kernel-trace profile of
# this tree's (eager) step.
#   bash scripts/gpu_calls/r6_ab.sh TAG "tests/test_a.py tests/test_b.py" [ROUNDS]
set -uo pipefail
TAG=${1:-r6ab}
SEL=${2:-tests/}
R=${3:-3}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
echo "== pytest $SEL"
timeout -k 10 600 python -u -m pytest --maxfail=10 -q --timeout 200 --timeout-method thread -m gpu $SEL > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -100; exit $rc; }
echo "== A/B headline"
bash scripts/ab_trees.sh $PWD/ab_old $PWD $R || exit 1
echo "== profile"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pbase -o p -- python3 bench.py --steps 10 --warmup 3 --graph 0 > $O/pbase.log 2>&1 || { tail -20 $O/pbase.log; exit 1; }
f=$(find $O/pbase -name "*kernel_stats.csv" | head -1)
python3 scripts/kstats.py "$f" 13 > $O/pbase.txt
head -30 $O/pbase.txt
