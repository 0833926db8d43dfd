#!/bin/bash
# A/B of the data-parallel eager step's host-side options on one GPU
# (--force-dp 1: single-rank RCCL communicator, collectives really issued).
set -uo pipefail
O=gpurun_out/dpab
mkdir -p $O
run() {
  name=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --steps 40 --warmup 10 --force-dp 1 > $O/$name.log 2>&1 || { tail -20 $O/$name.log; exit 1; }
  echo "$name $(tail -1 $O/$name.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
}
run base TDG_X=0
run nochunk TDG_DP_CHUNKED_WGRAD=0
run opt0 TDG_DP_OVERLAP_OPT=0
run nochunk_opt0 TDG_DP_CHUNKED_WGRAD=0 TDG_DP_OVERLAP_OPT=0
run graph TDG_DP_GRAPH=1
run base2 TDG_X=0
