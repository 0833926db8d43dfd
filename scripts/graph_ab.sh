#!/bin/bash
# Interleaved A/B: single-GPU step as a HIP graph vs eager (bench.py --graph).
set -uo pipefail
O=gpurun_out/graphab
mkdir -p $O
for r in 1 2 3; do
  for gr in 1 0; do
    timeout -k 10 240 python -u bench.py --steps 100 --warmup 20 --graph $gr > $O/g${gr}_$r.log 2>&1 || { tail -20 $O/g${gr}_$r.log; exit 1; }
    echo "graph=$gr run=$r $(tail -1 $O/g${gr}_$r.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step"
  done
done
