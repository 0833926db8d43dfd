set -uo pipefail
O=gpurun_out/c4; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fp8.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -60; exit $rc; }
timeout -k 10 300 python -u scripts/fp8_drelu_lab.py > $O/drelu.txt 2>&1 || exit 1
grep "round 1" $O/drelu.txt
timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 > $O/b8.log 2>&1 || exit 1
python -c "import json;d=[json.loads(l) for l in open('$O/b8.log') if l.startswith('{')][0];print('fp8 lean', d['ms_per_step'], d['config']['last_loss'])"
