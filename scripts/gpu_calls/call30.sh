set -uo pipefail
O=gpurun_out/c30; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp8.py -k "attn or attention" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -2 $O/t.txt
for r in 1 2; do
  for side in new old; do
    if [ $side = old ]; then export TDG_PKG_ROOT=ab_old; else unset TDG_PKG_ROOT; fi
    timeout -k 10 120 python3 -u scripts/attn_bench.py > $O/ab_$side$r.txt 2>&1 || { cat $O/ab_$side$r.txt; exit 1; }
    ATTN_B=16 ATTN_H=16 ATTN_L=512 timeout -k 10 120 python3 -u scripts/attn_bench.py >> $O/ab_$side$r.txt 2>&1 || { cat $O/ab_$side$r.txt; exit 1; }
    echo "== $side $r"; grep -v amdgpu.ids $O/ab_$side$r.txt
  done
done
unset TDG_PKG_ROOT
for r in 1 2; do
  for side in new old; do
    if [ $side = old ]; then export TDG_PKG_ROOT=ab_old; else unset TDG_PKG_ROOT; fi
    timeout -k 10 300 python3 -u scripts/ab_run.py -- --steps 40 --warmup 10 > $O/b_$side$r.log 2>&1 || { tail -20 $O/b_$side$r.log; exit 1; }
    echo "base $side $r: $(grep '^{' $O/b_$side$r.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])')"
  done
done
