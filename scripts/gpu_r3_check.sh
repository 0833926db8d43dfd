#!/bin/bash
# One GPU call: smoke, pytest -m gpu, the headline bench, the big-preset
# benches (BASELINE configs 4/5 per GPU) and kernel-trace profiles of the base
# and big-seq512-fp8 steps (library-kernel check). Every step time-limited;
# the script stops at the first failure.
set -uo pipefail
O=gpurun_out/${1:-r3check}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local n=$1 t=$2; shift 2; local rc; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; if [ $rc -ne 0 ]; then echo "$n failed rc=$rc"; tail -40 $O/$n.log; exit 1; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $O/pytest.log
step bench 300 python -u bench.py --steps 30 --warmup 10
tail -1 $O/bench.log
bn() { local n=$1; shift; step $n 400 python -u bench.py --steps 20 --warmup 5 "$@"; echo "$n $(grep '"metric"' $O/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; }
bn big --preset big
bn big512 --preset big --seq-len 512 --local-batch 16
bn big512_fp8 --preset big --seq-len 512 --local-batch 16 --dtype fp8
prof() { local n=$1; shift; mkdir -p $O/prof_$n; step prof_$n 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 bench.py --steps 8 --warmup 3 --graph 0 "$@"; python3 scripts/prof_summary.py $O/prof_$n > $O/prof_$n/summary.txt; head -8 $O/prof_$n/summary.txt; }
prof base
prof big --preset big
prof big512_fp8 --preset big --seq-len 512 --local-batch 16 --dtype fp8
