#!/bin/bash
# Counters of the ragged weight-gradient launch alone (one counter group per
# pass, --kernel-trace only) and the list of counters this box offers.
set -uo pipefail
TAG=${1:-r6wpmc}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -c "" $O/counters.txt
n=1
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o p$n --pmc $grp \
    -- python3 scripts/wgrad_ragged_run.py > $O/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/p$n.log; exit 1; }
  n=$((n+1))
done
python3 scripts/pmc_summary.py $O gemm256 > $O/summary.txt 2>&1
cat $O/summary.txt | head -40
python3 scripts/l2_table.py $O gemm256 | head -5
