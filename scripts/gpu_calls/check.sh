#!/bin/bash
# Round check on one MI355X: GPU tests, benches, kernel-trace profiles.
#   bash scripts/gpu_calls/check.sh [tag] [pytest selection...]
set -uo pipefail
TAG=${1:-check}
shift || true
SEL=${*:-tests/}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
step() { echo "== $1"; }
bench() {  # name, timeout, args...
  local n=$1 t=$2
  shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.log 2>&1 || { tail -30 $O/$n.log; exit 1; }
  python -c "import json;d=[json.loads(l) for l in open('$O/$n.log') if l.startswith('{')][0];print('$n', d['ms_per_step'], d['value'], d['config']['last_loss'])"
}
if [ "$SEL" != "none" ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu $SEL > $O/pytest.log 2>&1
  rc=$?
  tail -3 $O/pytest.log
  [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -80; exit $rc; }
fi
step bench
bench base1 300
bench base2 300
bench big 300 --preset big --steps 20 --warmup 5
bench big512_bf16 300 --preset big --seq-len 512 --local-batch 16 --steps 20 --warmup 5
bench big512_fp8 300 --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5
step profile
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pbase -o p -- python3 bench.py --steps 10 --warmup 3 --graph 0 > $O/pbase.log 2>&1 || { tail -20 $O/pbase.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p8 -o p -- python3 bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 10 --warmup 3 --graph 0 > $O/p8.log 2>&1 || { tail -20 $O/p8.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pbig -o p -- python3 bench.py --preset big --steps 10 --warmup 3 --graph 0 > $O/pbig.log 2>&1 || { tail -20 $O/pbig.log; exit 1; }
for d in pbase p8 pbig; do
  f=$(find $O/$d -name "*kernel_stats.csv" | head -1)
  python3 scripts/kstats.py "$f" 13 > $O/$d.txt
  head -30 $O/$d.txt
  t=$(find $O/$d -name "*kernel_trace.csv" | head -1)
  python3 scripts/ktrace_order.py "$t" 2 > $O/${d}_order.txt
done
