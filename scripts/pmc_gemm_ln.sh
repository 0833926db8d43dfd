#!/bin/bash
# L2 / wait counters of the fused projection+LayerNorm kernel vs the unfused
# GEMM (counters with --kernel-trace only; one counter group per pass).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/pmc_gemm_ln
mkdir -p $OUT
for K in 512 2048; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/l2_$K -o l2 \
    --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -- python3 scripts/gemm_ln_one.py --K $K --reps 20 > $OUT/l2_$K.log 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d $OUT/sq_$K -o sq \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 scripts/gemm_ln_one.py --K $K --reps 20 > $OUT/sq_$K.log 2>&1
done
for d in $OUT/*/; do echo "== $d"; python3 scripts/pmc_summary.py $d; done > $OUT/summary.txt 2>&1 || true
