#!/bin/bash
# Adam kernel change: numerics tests, then a kernel-trace profile of the step.
set -uo pipefail
O=gpurun_out/adam
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "adam or model or dp or graph" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash scripts/profile_bench.sh adam > /dev/null || exit 1
grep -i "adam\|last" gpurun_out/prof_adam/summary.txt
tail -1 gpurun_out/prof_adam/bench.log
