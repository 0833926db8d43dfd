set -uo pipefail
O=gpurun_out/c32; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp8.py > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
timeout -k 10 600 python3 -u scripts/gemm_vs_blas.py --preset big --cfgs 0,4,9,10,12,13,20,21,22 > $O/big.txt 2>&1 || { tail -20 $O/big.txt; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/c32/big.txt'):
    if not l.startswith('{'): continue
    d=json.loads(l)
    if 'total_us' in d: print(d); continue
    print(f"{d['kind']:6s} {d['name']:6s} {d['M']}x{d['N']}x{d['K']} blas {d['blas_us']:7.1f}  best cfg{d['best']} {d['best_us']:7.1f}  ratio {d['best_us']/d['blas_us']:.2f}")
PY
run() { n=$1; shift; timeout -k 10 300 python3 -u scripts/ab_run.py -- "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])')"; }
for r in 1 2; do
  unset TDG_PKG_ROOT; run base_new$r --steps 40 --warmup 10
  export TDG_PKG_ROOT=ab_old; run base_old$r --steps 40 --warmup 10
  unset TDG_PKG_ROOT; run big_new$r --preset big --steps 20 --warmup 5
  export TDG_PKG_ROOT=ab_old; run big_old$r --preset big --steps 20 --warmup 5
  unset TDG_PKG_ROOT; run f8_new$r --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5
  export TDG_PKG_ROOT=ab_old; run f8_old$r --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5
done
