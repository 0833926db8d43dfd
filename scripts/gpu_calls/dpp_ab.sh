#!/bin/bash
# DPP / permlane wave reductions: the kernel tests that use them, then an
# interleaved headline A/B against the previous build (ab_old/)
set -uo pipefail
T=${1:-dpp}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_ln_keep_bits.py tests/test_gpu_model.py \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
bash scripts/ab_trees.sh ab_old . 3 || exit 1
