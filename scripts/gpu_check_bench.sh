#!/bin/bash
# GPU tests (kernels, model, graph) then the headline bench twice.
set -uo pipefail
O=gpurun_out/${1:-chk}
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 > $O/bench_$r.log 2>&1 || { tail -20 $O/bench_$r.log; exit 1; }
  echo "bench $r: $(tail -1 $O/bench_$r.log | cut -c1-190)"
done
