#!/bin/bash
# In-model GEMM tile re-tune with HIP-graph timing (scripts/tune_in_model.py --graph 1).
#   bash scripts/gpu_calls/r6_tune.sh PRESET "CANDS"
set -uo pipefail
P=${1:-base}
C=${2:-4,9,10,12,13,20,22}
O=gpurun_out/tune
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
timeout -k 10 1000 python -u scripts/tune_in_model.py --preset $P --graph 1 --cands $C --rounds 3 --steps 20 ${TUNE_ARGS:-} --out $O/$P${TAG:-}.json 2>&1 | tee $O/$P${TAG:-}.log
