#!/bin/bash
# Eight gloo ranks on one MI355X, Transformer-base, with the host comm thread
# forced on so the segmented graph issues every span through the stream
# signal (ops/kernels.StreamSignal): replicas verified bitwise after the timed
# steps. Not a scaling measurement (eight ranks share one card).
set -uo pipefail
O=gpurun_out/r6dp8sig
mkdir -p $O
export TDG_NO_AUTOBUILD=1
( while sleep 45; do echo "[tick] $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK 2>/dev/null" EXIT
GPU_MAX_HW_QUEUES=1 TDG_DIST_BACKEND=gloo TDG_DP_COMM_THREAD=force timeout -k 10 900 python -u bench.py --gpus 8 --steps 6 --warmup 2 --verify-replicas 1 \
  > $O/dp8.log 2>&1
rc=$?
grep -E "dp_mode_select|^\{" $O/dp8.log | cut -c1-900
[ $rc -eq 0 ] || { tail -40 $O/dp8.log; exit $rc; }
