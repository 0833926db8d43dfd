#!/bin/bash
# One GPU call: kernel/model tests, then the headline bench in its variants.
set -uo pipefail
O=gpurun_out/check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 > $O/bench_graph.log 2>&1 || { tail -30 $O/bench_graph.log; exit 1; }
tail -1 $O/bench_graph.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --graph 0 > $O/bench_eager.log 2>&1 || { tail -30 $O/bench_eager.log; exit 1; }
tail -1 $O/bench_eager.log
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --force-dp 1 > $O/bench_dp1.log 2>&1 || { tail -30 $O/bench_dp1.log; exit 1; }
tail -1 $O/bench_dp1.log
