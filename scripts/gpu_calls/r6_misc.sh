#!/bin/bash
# Round-6 measurements on one MI355X: variable-length text training vs
# synthetic at the matched mean shape (HIP-graph bucket cache), then the
# in-tree vs hipBLASLt GEMM tables.
set -uo pipefail
TAG=${1:-r6misc}; SCHEDS=${2:-"cur"}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
echo "== text vs synthetic"
timeout -k 10 600 python -u scripts/text_vs_synthetic.py > $O/text_vs_synth.log 2>&1 || { tail -30 $O/text_vs_synth.log; exit 1; }
grep '^{' $O/text_vs_synth.log
bash scripts/gpu_calls/r6_blas.sh $TAG "$SCHEDS"
