#!/bin/bash
# A/B of the manual-GC policy (utils/gcpolicy.py) on the eager data-parallel
# step (--force-dp 1) and the single-GPU graph step, interleaved runs.
set -uo pipefail
O=gpurun_out/gcab
mkdir -p $O
run() {
  name=$1; gcv=$2; shift 2
  TDG_MANUAL_GC=$gcv timeout -k 10 240 python -u bench.py --steps 60 --warmup 10 "$@" > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name $(tail -1 $O/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
for r in 1 2 3; do
  run dp_gc0_$r 0 --force-dp 1
  run dp_gc1_$r 1 --force-dp 1
done
run graph_gc1 1
run eager_gc1 1 --graph 0
