#!/bin/bash
# Interleaved A/B of bench.py under environment variants.
#   bash scripts/ab_env.sh TAG ROUNDS "ENV=a ENV2=b" "ENV=c" ...   ("-" = no extra env)
# Prints ms/step per (variant, round); logs under gpurun_out/ab_TAG/.
set -uo pipefail
TAG=$1; R=$2; shift 2
O=gpurun_out/ab_$TAG
mkdir -p $O
BARGS=${BENCH_ARGS:---steps 60 --warmup 15}
for r in $(seq 1 $R); do
  i=0
  for v in "$@"; do
    i=$((i+1))
    ev=""; [ "$v" != "-" ] && ev="$v"
    env $ev timeout -k 10 300 python -u bench.py $BARGS > $O/v${i}_$r.log 2>&1 || { echo "variant $i ($v) failed"; tail -20 $O/v${i}_$r.log; exit 1; }
    echo "[$v] run=$r $(tail -1 $O/v${i}_$r.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step"
  done
done
