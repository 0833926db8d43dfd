#!/bin/bash
# attention kernel tests, PMC of the base step's attention kernels, and an
# interleaved headline A/B against the previous build (ab_old/)
set -uo pipefail
T=${1:-abat}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "attn or attention" \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for t in ab_old .; do
  n=$(basename $(cd $t && pwd))
  (cd $t && timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $PWD/gpurun_out/$T/pmc_$n -o p \
    --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES \
    -- python3 scripts/attn_one.py > /dev/null 2>&1) || { echo "pmc $t failed"; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/$T/pmc_$n attn_bwd_fused | head -6
done
bash scripts/ab_trees.sh ab_old . 3 || exit 1
