#!/bin/bash
# LayerNorm backward at d_model 512: 2 rows per wave (this tree) against 4
# (ab_old/), with 32 and 16 rows per workgroup (TDG_LN_BWD_RPB), interleaved.
set -uo pipefail
export TDG_NO_AUTOBUILD=1
O=$PWD/gpurun_out/r6lnrpw
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "ln or layernorm" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
  for v in old new32 new16; do
    case $v in
      old) d=$PWD/ab_old; e="";;
      new32) d=$PWD; e="TDG_LN_BWD_RPB=32";;
      new16) d=$PWD; e="TDG_LN_BWD_RPB=16";;
    esac
    (cd $d && env $e timeout -k 10 300 python -u bench.py --steps 60 --warmup 15 > $O/${v}_$r.log 2>&1) || { echo "$v failed"; tail -5 $O/${v}_$r.log; exit 1; }
    echo "[$v] run=$r $(tail -1 $O/${v}_$r.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step"
  done
done
