#!/bin/bash
# L2 counters of every kernel of config 5 (Transformer-big, seq 512, fp8)
# eager steps, incl. the fp8 weight-gradient launch: TCC hits / misses /
# fabric read requests in one pass, FETCH_SIZE in another (--kernel-trace
# only, one counter group per pass); table by scripts/l2_table.py.
set -uo pipefail
O=gpurun_out/r6l2fp8
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
A="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 2 --warmup 1 --graph 0"
n=1
for grp in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" "FETCH_SIZE"; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o p$n --pmc $grp \
    -- python3 bench.py $A > $O/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/p$n.log; exit 1; }
  n=$((n+1))
done
python3 scripts/l2_table.py $O > $O/l2.txt 2>&1
head -30 $O/l2.txt
