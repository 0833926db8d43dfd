set -uo pipefail
O=gpurun_out/c50; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_kernels.py tests/test_gpu_model.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for r in 1 2; do
  for side in new old; do
    if [ $side = old ]; then export TDG_PKG_ROOT=ab_old; else unset TDG_PKG_ROOT; fi
    echo "== $side $r"; timeout -k 10 120 python3 -u scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids
  done
done
run() { n=$1; shift; timeout -k 10 300 python3 -u scripts/ab_run.py -- "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])')"; }
F8="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5"
for r in 1 2; do
  unset TDG_PKG_ROOT; run base_new$r --steps 40 --warmup 10
  export TDG_PKG_ROOT=ab_old; run base_old$r --steps 40 --warmup 10
  unset TDG_PKG_ROOT; run big_new$r --preset big --steps 20 --warmup 5
  export TDG_PKG_ROOT=ab_old; run big_old$r --preset big --steps 20 --warmup 5
  unset TDG_PKG_ROOT; run f8_new$r $F8
  export TDG_PKG_ROOT=ab_old; run f8_old$r $F8
done
