#!/bin/bash
# BASELINE configs 4 and 5 on one GPU (per-GPU work of the DP=8 runs):
# Transformer-big seq 128 batch 64 bf16; big seq 512 batch 16 bf16 and fp8.
set -uo pipefail
O=gpurun_out/big
mkdir -p $O
run() { n=$1; shift; timeout -k 10 400 python -u bench.py --steps 30 --warmup 10 "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; echo "$n $(grep '"metric"' $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; }
run big --preset big
run big512 --preset big --seq-len 512 --local-batch 16
run big512_fp8 --preset big --seq-len 512 --local-batch 16 --dtype fp8
run big_dp1 --preset big --force-dp 1
