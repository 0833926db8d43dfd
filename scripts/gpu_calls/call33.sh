set -uo pipefail
O=gpurun_out/c33; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
a="--preset big --seq-len 512 --local-batch 16 --dtype fp8"
for side in new old; do
  if [ $side = old ]; then export TDG_PKG_ROOT=ab_old; else unset TDG_PKG_ROOT; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$side -o p -- python3 scripts/ab_run.py -- $a --steps 10 --warmup 3 --graph 0 > $O/$side.log 2>&1 || { tail -20 $O/$side.log; exit 1; }
done
python3 scripts/kstats_diff.py $(find $O/new -name "*kernel_stats.csv" | head -1) $(find $O/old -name "*kernel_stats.csv" | head -1) 13
