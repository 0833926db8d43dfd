#!/bin/bash
# Stream-signal issue path: GPU tests (signal + DP rehearsals) and the
# one-rank DP step with the signal (default) vs the event cut, plus the
# single graph, interleaved.
set -uo pipefail
O=gpurun_out/r6sig
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_signal.py tests/test_gpu_dp.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for v in sig ev one; do
    case $v in
      sig) E="TDG_DP_SIGNAL=1"; A="--force-dp 1";;
      ev)  E="TDG_DP_SIGNAL=0"; A="--force-dp 1";;
      one) E="TDG_DP_SIGNAL=1"; A="";;
    esac
    env $E timeout -k 10 200 python3 bench.py $A --steps 100 --warmup 20 > $O/b_${v}_$r.log 2>&1 || { tail -20 $O/b_${v}_$r.log; exit 1; }
    echo "$v r$r $(grep '^{' $O/b_${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("dp_mode_select",""))')"
  done
done
