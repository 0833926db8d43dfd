#!/bin/bash
# Data-parallel step (single RCCL rank, segmented HIP graph) option sweep:
# per-span Adam placement and span size; graph single-GPU step as reference.
set -uo pipefail
O=gpurun_out/dpsweep
mkdir -p $O
run() { n=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --force-dp 1 $EXTRA > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; echo "$n $(tail -1 $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])') $(grep spans $O/$n.log | cut -c48-)"; }
EXTRA="" run tail64 TDG_DP_OVERLAP_OPT=tail
EXTRA="" run opt0_64 TDG_DP_OVERLAP_OPT=0
EXTRA="--bucket-mb 128" run tail128 TDG_DP_OVERLAP_OPT=tail
EXTRA="--bucket-mb 32" run tail32 TDG_DP_OVERLAP_OPT=tail
EXTRA="--bucket-mb 512" run tail512 TDG_DP_OVERLAP_OPT=tail
EXTRA="" run nochunk TDG_DP_CHUNKED_WGRAD=0
timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 > $O/single.log 2>&1 && echo "single $(tail -1 $O/single.log | cut -c150-175)"
