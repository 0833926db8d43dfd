#!/bin/bash
# config-5 kernel stats with the persistent fp8 GEMM off / on
set -uo pipefail
T=${1:-pkprof}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for p in 0 1; do
  TDG_FP8_PERSIST=$p timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$p -o p -- python3 bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 10 --warmup 3 --graph 0 > $O/p$p.log 2>&1 || { tail -20 $O/p$p.log; exit 1; }
  f=$(find $O/p$p -name "*kernel_stats.csv" | head -1)
  python3 scripts/kstats.py "$f" 13 > $O/p$p.txt
done
python3 scripts/kstats_diff.py $(find $O/p1 -name "*kernel_stats.csv" | head -1) $(find $O/p0 -name "*kernel_stats.csv" | head -1) 13 | head -25
