#!/bin/bash
# PMC comparison of several GEMM configs on one shape.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/pmc_multi; mkdir -p $OUT
SHAPE="$1"; shift
for cfg in "$@"; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/c${cfg}a -o a --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -- python3 scripts/gemm_one.py $SHAPE --cfg $cfg --reps 20 > /dev/null 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/c${cfg}b -o b --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA -- python3 scripts/gemm_one.py $SHAPE --cfg $cfg --reps 20 > /dev/null 2>&1 || \
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/c${cfg}b -o b --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU -- python3 scripts/gemm_one.py $SHAPE --cfg $cfg --reps 20 > /dev/null 2>&1
  python3 scripts/gemm_one.py $SHAPE --cfg $cfg --reps 50
  echo "== cfg$cfg"; python3 scripts/pmc_summary.py $OUT/c${cfg}a gemm_kernel | tail -n +2; python3 scripts/pmc_summary.py $OUT/c${cfg}b gemm_kernel | tail -n +2
done
