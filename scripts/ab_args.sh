#!/bin/bash
# Interleaved A/B of bench.py argument/env variants (one box, one process per run).
#   bash scripts/ab_args.sh TAG ROUNDS "ENV=a|--arg x" "-|--force-dp 1" ...
# Each variant is "ENV ASSIGNMENTS|BENCH ARGS" ("-" = none on that side).
set -uo pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/ab_$TAG
mkdir -p $O
BASE=${BENCH_ARGS:---steps 60 --warmup 15}
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    ev=${v%%|*}; av=${v#*|}
    [ "$ev" = "-" ] && ev=""
    [ "$av" = "-" ] && av=""
    env $ev timeout -k 10 300 python -u bench.py $BASE $av > $O/v${i}_$r.log 2>&1 || { echo "variant $i ($v) failed"; tail -20 $O/v${i}_$r.log; exit 1; }
    echo "[$v] run=$r $(tail -1 $O/v${i}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("hip_graph"))') ms/step"
  done
done
