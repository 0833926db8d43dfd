#!/bin/bash
# Round-2 GEMM epilogue rework: GPU tests, the step bench with the current
# tuned table, an in-model re-tune, and the bench with the re-tuned table.
set -uo pipefail
O=gpurun_out/r2g
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $O/bench_old_table.log 2>&1 || { tail -20 $O/bench_old_table.log; exit 1; }
echo "old table: $(tail -1 $O/bench_old_table.log | cut -c1-200)"
timeout -k 10 600 python -u scripts/tune_in_model.py --preset base --out $O/tuned_inmodel.json > $O/tune.log 2>&1 || { tail -20 $O/tune.log; exit 1; }
tail -3 $O/tune.log
TDG_GEMM_TUNED_FILE=$O/tuned_inmodel.json timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $O/bench_new_table.log 2>&1 || { tail -20 $O/bench_new_table.log; exit 1; }
echo "new table: $(tail -1 $O/bench_new_table.log | cut -c1-200)"
