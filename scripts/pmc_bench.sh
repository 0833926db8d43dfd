#!/bin/bash
# PMC counters for every kernel of a few eager training steps of the headline
# bench (counters only with --kernel-trace; one counter group per pass) and a
# per-kernel table (scripts/pmc_table.py).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/pmc_bench${PMC_TAG:-}
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p1 -o p1 \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -- python3 bench.py --steps 3 --warmup 2 --graph 0 "$@" > $OUT/p1.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p2 -o p2 \
  --pmc FETCH_SIZE -- python3 bench.py --steps 3 --warmup 2 --graph 0 "$@" > $OUT/p2.log 2>&1
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/p3 -o p3 \
  --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA \
  -- python3 bench.py --steps 3 --warmup 2 --graph 0 "$@" > $OUT/p3.log 2>&1
python3 scripts/pmc_table.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
