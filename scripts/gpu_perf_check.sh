#!/bin/bash
# One GPU call, performance only: the headline bench, the big-preset benches
# (BASELINE configs 4/5 per GPU) and kernel-trace profiles of the base and big
# steps. Every step time-limited; the script stops at the first failure.
set -uo pipefail
O=gpurun_out/${1:-perf}
mkdir -p $O
export TMPDIR=/tmp
step() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; if [ $rc -ne 0 ]; then echo "$n failed rc=$rc"; tail -40 $O/$n.log; exit 1; fi; }
bn() { n=$1; shift; step $n 400 python -u bench.py --steps 30 --warmup 10 "$@"; echo "$n $(grep '"metric"' $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; }
bn base
bn big --preset big
bn big512 --preset big --seq-len 512 --local-batch 16
bn big512_fp8 --preset big --seq-len 512 --local-batch 16 --dtype fp8
prof() { n=$1; shift; mkdir -p $O/prof_$n; step prof_$n 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 bench.py --steps 8 --warmup 3 --graph 0 "$@"; }
prof base
prof big --preset big
