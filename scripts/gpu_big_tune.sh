#!/bin/bash
# Transformer-big in-model GEMM re-tune (round-2 epilogue) and the benches
# with the re-tuned table.
set -uo pipefail
O=gpurun_out/bigtune
mkdir -p $O
timeout -k 10 900 python -u scripts/tune_in_model.py --preset big --out $O/tuned_big.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -1 $O/tune.log
for v in "big:--preset big" "big512:--preset big --seq-len 512 --local-batch 16"; do
  n=${v%%:*}; a=${v#*:}
  TDG_GEMM_TUNED_FILE=$O/tuned_big.json timeout -k 10 400 python -u bench.py --steps 30 --warmup 10 $a > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  echo "$n $(grep '"metric"' $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
