#!/bin/bash
# Kernel traces of the one-rank data-parallel step (--force-dp 1) and the
# single graph, per-kernel tables side by side.
set -uo pipefail
O=gpurun_out/r6dpprof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
for v in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$v -o p -- python3 bench.py --force-dp $v --steps 20 --warmup 10 > $O/p$v.log 2>&1 || { tail -20 $O/p$v.log; exit 1; }
  f=$(find $O/p$v -name "*kernel_stats.csv" | head -1)
  python3 scripts/kstats.py "$f" 33 > $O/p$v.txt
done
python3 scripts/kstats_diff.py $(find $O/p0 -name "*kernel_stats.csv" | head -1) $(find $O/p1 -name "*kernel_stats.csv" | head -1) 33 > $O/diff.txt 2>&1 || true
head -3 $O/p0.txt; head -3 $O/p1.txt; head -30 $O/diff.txt
