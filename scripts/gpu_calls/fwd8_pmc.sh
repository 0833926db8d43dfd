#!/bin/bash
# PMC counters of the e4m3 attention forward (lab shape; counters with
# --kernel-trace only, one counter group per pass)
set -uo pipefail
T=${1:-fwd8pmc}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/p1 -o p1 \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS \
  -- python3 scripts/attn_fwd8_lab.py > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $O/p2 -o p2 \
  --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM \
  -- python3 scripts/attn_fwd8_lab.py > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
python3 scripts/pmc_summary.py $O attn_fwd_fp8 > $O/summary.txt
cat $O/summary.txt
