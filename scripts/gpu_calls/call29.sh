set -uo pipefail
O=gpurun_out/c29; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
run() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.log 2>&1 || { tail -30 $O/$n.log; exit 1; }; python -c "import json;d=[json.loads(l) for l in open('$O/$n.log') if l.startswith('{')][0];print('$n', d['ms_per_step'], d['value'], d['config']['last_loss'])"; }
run base1 && run base2 && run big1 --preset big --steps 20 --warmup 5 && \
run b8a --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 && \
run b16 --preset big --seq-len 512 --local-batch 16 --steps 20 --warmup 5
timeout -k 10 120 python -u bench.py --gpus 2 > $O/g2.log 2>&1; echo "bench --gpus 2 on one GPU exit: $? (expected 2)"; tail -2 $O/g2.log
