set -uo pipefail
O=gpurun_out/c34; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py -k "attention" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
run() { n=$1; shift; timeout -k 10 300 python3 -u scripts/ab_run.py "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }; echo "$n $(grep '^{' $O/$n.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read())["ms_per_step"])')"; }
F8="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5"
for r in 1 2; do
  run with10_$r -- $F8
  run no10_$r ops.fp8._CANDS=0,1,2,3,4,5,8,9 -- $F8
done
