#!/bin/bash
# config-4 (Transformer-big, seq 128, bf16) kernel stats
set -uo pipefail
T=${1:-pbig}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o p -- python3 bench.py --preset big --steps 10 --warmup 3 --graph 0 > $O/p.log 2>&1 || { tail -20 $O/p.log; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
python3 scripts/kstats.py "$f" 13 > $O/p.txt
head -30 $O/p.txt
