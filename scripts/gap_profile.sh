#!/bin/bash
# Kernel trace of the GRAPH-replayed step (single graph and the segmented
# data-parallel graph on one rank) and its idle-gap summary.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in "single:" "dpseg:--force-dp 1"; do
  n=${v%%:*}; a=${v#*:}
  OUT=gpurun_out/gaps_$n
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT -o run -- python3 bench.py --steps 12 --warmup 3 $a > $OUT/bench.log 2>&1
  python3 scripts/gap_summary.py $OUT > $OUT/gaps.txt
  cat $OUT/gaps.txt
done
