#!/bin/bash
# One GPU call: smoke, pytest -m gpu, the headline bench. Every step
# time-limited; the script stops at the first failure.
set -uo pipefail
O=gpurun_out/${1:-r4check}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
step() { local n=$1 t=$2; shift 2; local rc; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; if [ $rc -ne 0 ]; then echo "$n failed rc=$rc"; tail -40 $O/$n.log; exit 1; fi; }
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
step pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -2 $O/pytest.log
step bench 300 python -u bench.py --steps 30 --warmup 10
tail -1 $O/bench.log
step bench2fail 120 bash -c "python -u bench.py --gpus 2 --steps 2 --warmup 1; test \$? -eq 2"
tail -2 $O/bench2fail.log
