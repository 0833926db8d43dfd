#!/bin/bash
# write-through attention / LayerNorm-copy / embedding outputs: kernel tests,
# then interleaved headline and config-5 A/Bs against ab_old/
set -uo pipefail
T=${1:-wt}
O=gpurun_out/$T
mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ \
  > $O/pytest.log 2>&1 || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit 1; }
tail -1 $O/pytest.log
bash scripts/ab_trees.sh ab_old . 3 || exit 1
for r in 1 2; do
  for t in ab_old .; do
    n=$(basename $(realpath $t))
    (cd $t && timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 > $OLDPWD/$O/f8_${n}_$r.log 2>&1) || { echo "$t fp8 failed"; exit 1; }
    echo "[fp8 $n] run=$r $(tail -1 $O/f8_${n}_$r.log | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step"
  done
done
