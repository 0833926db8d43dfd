#!/bin/bash
# Kernel trace of the one-rank DP step with the stream signal (default) and
# with the event cut (TDG_DP_SIGNAL=0): per-step gaps.
set -uo pipefail
O=gpurun_out/r6sigprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
for v in ${SIGS:-1 0}; do
  export TDG_DP_SIGNAL=$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$v -o p -- python3 bench.py --force-dp 1 --steps 20 --warmup 10 > $O/s$v.log 2>&1 || { tail -20 $O/s$v.log; exit 1; }
  f=$(find $O/s$v -name "*kernel_trace.csv" | head -1)
  echo "== TDG_DP_SIGNAL=$v  $(grep -o '"ms_per_step": [0-9.]*' $O/s$v.log)"
  python3 scripts/gap_report.py "$f" 3
  grep -h "signal" $(find $O/s$v -name "*kernel_stats.csv") | cut -c1-160 || true
  rm -f "$f"
done
