#!/bin/bash
# scripts/ln_fused_lab.py on one MI355X (fused post-LN epilogue ablations)
set -uo pipefail
O=gpurun_out/lnlab
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python -u scripts/ln_fused_lab.py 2>&1 | tee $O/lab.txt
