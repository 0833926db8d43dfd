#!/bin/bash
# Fused post-LN GEMM epilogues: numerics tests, interleaved A/B of the
# headline step with / without them, kernel trace of the fused step.
set -uo pipefail
O=gpurun_out/lnf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread ${LNF_TESTS:-tests/test_gpu_ln_fused.py} > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $O/pytest.log | head -120; exit $rc; }
timeout -k 10 300 python -u scripts/ln_fused_lab.py > $O/lab.txt 2>&1 || { tail -20 $O/lab.txt; exit 1; }
cat $O/lab.txt
bash scripts/ab_env.sh lnf ${ROUNDS:-3} "TDG_LN_KEEP_BITS=0" "-" "TDG_LN_FUSED=bwd" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 bench.py --steps 10 --warmup 3 --graph 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 scripts/kstats.py "$f" 13 > $O/kstats.txt
head -30 $O/kstats.txt
t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 scripts/ktrace_order.py "$t" 2 > $O/order.txt
tail -3 $O/order.txt
