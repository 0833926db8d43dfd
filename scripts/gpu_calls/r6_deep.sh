#!/bin/bash
# gemm256 two-ahead half-tile refill (TDG_G256_DEEP): GPU GEMM / model /
# graph tests, the ragged weight-gradient lab with it off / on, headline and
# config-4 A/Bs, and the L2 counters of the eager headline step with it on.
set -uo pipefail
TAG=${1:-r6deep}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
echo "== pytest"
timeout -k 10 600 python -u -m pytest --maxfail=10 -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_graph.py tests/test_gpu_text_graph.py tests/test_gpu_model.py \
  tests/test_gpu_fp8.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -120; exit $rc; }
echo "== wgrad lab"
for d in 0 1; do
  TDG_G256_DEEP=$d CFGS=12 timeout -k 10 300 python -u scripts/wgrad_lab.py > $O/lab_deep$d.txt 2>&1 || { tail -20 $O/lab_deep$d.txt; exit 1; }
  grep "ragged" $O/lab_deep$d.txt | sed "s/^/deep=$d /"
done
echo "== A/B headline"
bash scripts/ab_env.sh deep_base 3 "TDG_G256_DEEP=0" "TDG_G256_DEEP=1" || exit 1
echo "== A/B big"
BENCH_ARGS="--preset big --steps 20 --warmup 5" bash scripts/ab_env.sh deep_big 2 "TDG_G256_DEEP=0" "TDG_G256_DEEP=1" || exit 1
echo "== L2 counters (deep)"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/l2a -o l2a \
  --pmc TCC_HIT_sum TCC_MISS_sum -- python3 bench.py --steps 3 --warmup 2 --graph 0 > $O/l2a.log 2>&1 || { tail -5 $O/l2a.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ks -o ks -- python3 bench.py --steps 10 --warmup 3 --graph 0 > $O/ks.log 2>&1 || { tail -5 $O/ks.log; exit 1; }
python3 scripts/l2_table.py $O > $O/l2_table.txt
head -12 $O/l2_table.txt
f=$(find $O/ks -name "*kernel_stats.csv" | head -1)
python3 scripts/kstats.py "$f" 13 > $O/kstats.txt
head -20 $O/kstats.txt
