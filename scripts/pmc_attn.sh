#!/bin/bash
# PMC counters for the attention kernels (counters with --kernel-trace only).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/${1:-pmc_attn}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -- python3 scripts/attn_one.py > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -- python3 scripts/attn_one.py > $OUT/p2.log 2>&1
python3 scripts/pmc_summary.py $OUT attn > $OUT/summary.txt
cat $OUT/summary.txt
