#!/bin/bash
# Round-6 check on one MI355X: the GPU test suite (or a selection), the
# headline bench twice, then L2 counters of the eager headline step (one
# counter group per pass, --kernel-trace only).
#   bash scripts/gpu_calls/r6_check.sh TAG [pytest selection | none]
set -uo pipefail
TAG=${1:-r6check}
shift || true
SEL=${*:-tests/}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
if [ "$SEL" != "none" ]; then
  echo "== pytest $SEL"
  timeout -k 10 900 python -u -m pytest --maxfail=15 -v --timeout 200 --timeout-method thread -m gpu $SEL > $O/pytest.log 2>&1
  rc=$?
  tail -3 $O/pytest.log
  [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert\|FAIL" $O/pytest.log | head -120; exit $rc; }
fi
for n in base1 base2; do
  timeout -k 10 300 python -u bench.py > $O/$n.log 2>&1 || { tail -30 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | cut -c1-200
done
[ "${PMC:-1}" = "1" ] || exit 0
echo "== L2 counters"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/l2a -o l2a \
  --pmc TCC_HIT_sum TCC_MISS_sum -- python3 bench.py --steps 3 --warmup 2 --graph 0 > $O/l2a.log 2>&1 || { tail -5 $O/l2a.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/l2b -o l2b \
  --pmc FETCH_SIZE -- python3 bench.py --steps 3 --warmup 2 --graph 0 > $O/l2b.log 2>&1 || { tail -5 $O/l2b.log; exit 1; }
python3 scripts/l2_table.py $O > $O/l2_table.txt
head -30 $O/l2_table.txt
