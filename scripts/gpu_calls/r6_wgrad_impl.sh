#!/bin/bash
# The ragged weight-gradient main loop: lock-step gemm256 (0) against the
# pipelined one-wave-per-SIMD loop with a 4 / 5-slot ring (1 / 2), in the
# headline step and in config 4, interleaved (TDG_WGRAD_IMPL).
set -uo pipefail
export TDG_NO_AUTOBUILD=1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k ragged > gpurun_out/wimpl_tests.log 2>&1; tail -2 gpurun_out/wimpl_tests.log
bash scripts/ab_env.sh wimpl 3 "TDG_WGRAD_IMPL=0" "TDG_WGRAD_IMPL=1" "TDG_WGRAD_IMPL=2" || exit 1
BENCH_ARGS="--preset big --steps 20 --warmup 5" bash scripts/ab_env.sh wimplbig 2 "TDG_WGRAD_IMPL=0" "TDG_WGRAD_IMPL=1" "TDG_WGRAD_IMPL=2"
