#!/bin/bash
set -uo pipefail
O=gpurun_out/ksweep
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python -u scripts/fp8_ksweep.py > $O/ksweep.log 2>&1 || { tail -20 $O/ksweep.log; exit 1; }
cat $O/ksweep.log
