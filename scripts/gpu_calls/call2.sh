set -uo pipefail
O=gpurun_out/c2; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_dp.py -k "fp8" > $O/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -70 > $O/pytest_summary.txt
tail -4 $O/pytest_summary.txt
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" $O/pytest.log | head -100; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 > $O/b8_$i.log 2>&1 || exit 1
python -c "import json;d=[json.loads(l) for l in open('$O/b8_$i.log') if l.startswith('{')][0];print('fp8 lean', d['ms_per_step'], d['config']['last_loss'])"
timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--preset','big','--seq-len','512','--local-batch','16','--dtype','fp8','--steps','20','--warmup','5']
from tensorflow_distributed_on_gke_amd.ops import fp8; fp8.WGRAD_FP8=False
import runpy; runpy.run_path('bench.py', run_name='__main__')" > $O/b8o_$i.log 2>&1 || exit 1
python -c "import json;d=[json.loads(l) for l in open('$O/b8o_$i.log') if l.startswith('{')][0];print('fp8 bf16-wgrad', d['ms_per_step'], d['config']['last_loss'])"
done
timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --steps 20 --warmup 5 > $O/b16.log 2>&1 || exit 1
python -c "import json;d=[json.loads(l) for l in open('$O/b16.log') if l.startswith('{')][0];print('bf16', d['ms_per_step'], d['config']['last_loss'])"
