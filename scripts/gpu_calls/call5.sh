set -uo pipefail
O=gpurun_out/c5; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 700 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_dp.py -k "fp8" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B10 -A40 "Error\|assert" $O/pytest.log | head -120; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 > $O/b8_$i.log 2>&1 || { tail -30 $O/b8_$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/b8_$i.log') if l.startswith('{')][0];print('fp8 lean attn', d['ms_per_step'], d['config']['last_loss'])"
timeout -k 10 300 python -u -c "
import sys; sys.argv=['bench.py','--preset','big','--seq-len','512','--local-batch','16','--dtype','fp8','--steps','20','--warmup','5']
from tensorflow_distributed_on_gke_amd.ops import fp8; fp8.ATTN_PROJ_FP8=False
import runpy; runpy.run_path('bench.py', run_name='__main__')" > $O/b8o_$i.log 2>&1 || exit 1
python -c "import json;d=[json.loads(l) for l in open('$O/b8o_$i.log') if l.startswith('{')][0];print('fp8 bf16 attn-proj', d['ms_per_step'], d['config']['last_loss'])"
done
