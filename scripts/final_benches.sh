#!/bin/bash
# Every BASELINE configuration that runs on one MI355X, back to back, one JSON
# line each (appended to $1). Each step under its own time limit; the script
# stops at the first failure.
set -e
out=${1:-gpurun_out/benches.jsonl}
mkdir -p "$(dirname "$out")"
run() { timeout -k 10 300 python bench.py "$@" 2>/dev/null | grep '^{' >> "$out"; }
run --steps 50 --warmup 10                                                 # config 2: base, headline
run --steps 50 --warmup 10 --force-dp 1                                    # the per-rank DP path
run --steps 30 --warmup 10 --grad-comm bf16 --force-dp 1                   # DP path, bf16 gradient comm
TDG_DP_GRAPH=1 run --steps 50 --warmup 10 --force-dp 1                     # DP path as a HIP graph (opt-in)
run --steps 30 --warmup 10 --preset big                                    # config 4 (per GPU)
run --steps 30 --warmup 10 --preset big --seq-len 512 --local-batch 16     # big seq 512 bf16
run --steps 30 --warmup 10 --preset big --seq-len 512 --local-batch 16 --dtype fp8  # config 5 (per GPU)
