#!/bin/bash
# Kernel traces (graph replay / eager) of the single-GPU step, the segmented
# data-parallel step and the eager data-parallel step on one rank; idle gaps
# and per-kernel busy time of each.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in "single::" "dpseg::--force-dp 1" "dpeager:TDG_DP_GRAPH=0:--force-dp 1"; do
  n=${v%%:*}; rest=${v#*:}; e=${rest%%:*}; a=${rest#*:}
  OUT=gpurun_out/gaps3_$n
  mkdir -p $OUT
  [ -n "$e" ] && export $e
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 12 --warmup 3 $a > $OUT/bench.log 2>&1
  [ -n "$e" ] && unset ${e%%=*}
  python3 scripts/gap_summary.py $OUT > $OUT/gaps.txt
  python3 scripts/prof_summary.py $OUT > $OUT/summary.txt
  echo "== $n"; head -8 $OUT/gaps.txt; head -3 $OUT/summary.txt | tail -2
done
