#!/bin/bash
# Segmented data-parallel graph + round-2 fixes: targeted GPU tests, smoke,
# then the bench single-GPU graph vs the data-parallel path (single RCCL rank)
# as segmented graph / eager.
set -uo pipefail
O=gpurun_out/seg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_dp.py "tests/test_gpu_kernels.py::test_prep_batch" \
  -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for v in "graph:" "dp_seg:--force-dp 1" "dp_eager:--force-dp 1 --graph 0" "dp_seg_bf16:--force-dp 1 --grad-comm bf16"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 $a > $O/bench_$n.log 2>&1 || { tail -30 $O/bench_$n.log; exit 1; }
  echo "$n $(tail -1 $O/bench_$n.log)"
done
