set -uo pipefail
O=gpurun_out/c45; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_model.py tests/test_gpu_graph.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
run() { n=$1; shift; timeout -k 10 300 python3 -u scripts/ab_run.py -- "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])')"; }
for r in 1 2; do
  unset TDG_PKG_ROOT; run base_new$r --steps 40 --warmup 10
  export TDG_PKG_ROOT=ab_old; run base_old$r --steps 40 --warmup 10
  unset TDG_PKG_ROOT; run big_new$r --preset big --steps 20 --warmup 5
  export TDG_PKG_ROOT=ab_old; run big_old$r --preset big --steps 20 --warmup 5
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for side in new old; do
  if [ $side = old ]; then export TDG_PKG_ROOT=ab_old; else unset TDG_PKG_ROOT; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$side -o p -- python3 scripts/ab_run.py -- --preset big --steps 10 --warmup 3 --graph 0 > $O/prof_$side.log 2>&1 || { tail -20 $O/prof_$side.log; exit 1; }
done
python3 scripts/kstats_diff.py $(find $O/new -name "*kernel_stats.csv" | head -1) $(find $O/old -name "*kernel_stats.csv" | head -1) 13 | head -12
