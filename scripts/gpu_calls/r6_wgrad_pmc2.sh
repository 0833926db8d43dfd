#!/bin/bash
# Memory-path counters of the ragged weight-gradient launch alone: texture
# addresser / data, L1 (TCP) stalls on L2 data, LDS FIFOs, L2 -> fabric reads
# (DRAM vs all), one counter group per pass (--kernel-trace only).
set -uo pipefail
TAG=${1:-r6wpmc2}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
n=1
for grp in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" \
           "TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INST_LEVEL_LDS SQ_INSTS_LDS" \
           "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum TCC_TAG_STALL_sum"; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/p$n -o p$n --pmc $grp \
    -- python3 scripts/wgrad_ragged_run.py > $O/p$n.log 2>&1 || { echo "pass $n failed"; tail -5 $O/p$n.log; exit 1; }
  n=$((n+1))
done
python3 scripts/pmc_summary.py $O gemm256 > $O/summary.txt 2>&1
cat $O/summary.txt | head -40
