#!/bin/bash
# Interleaved bench.py A/B of two source trees on one box (each tree with its
# own in-tree built extensions): bash scripts/ab_trees.sh TREE_A TREE_B ROUNDS
set -uo pipefail
A=$1; B=$2; R=${3:-3}
O=$PWD/gpurun_out/ab_trees
mkdir -p $O
for r in $(seq 1 $R); do
  for t in "$A" "$B"; do
    n=$(basename "$t")
    (cd "$t" && timeout -k 10 300 python -u bench.py ${BENCH_ARGS:---steps 60 --warmup 15} > $O/${n}_$r.log 2>&1) || { echo "$t failed"; tail -5 $O/${n}_$r.log; exit 1; }
    echo "[$n] run=$r $(tail -1 $O/${n}_$r.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step"
  done
done
