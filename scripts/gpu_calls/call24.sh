set -uo pipefail
O=gpurun_out/c24; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dp.py tests/test_gpu_model.py tests/test_gpu_graph.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
for v in 0 1; do
timeout -k 10 300 python -u scripts/ab_run.py train.optim.ADAM_CHUNKED=$v -- --force-dp 1 > $O/d$v$i.log 2>&1 || { tail -30 $O/d$v$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/d$v$i.log') if l.startswith('{')][0];print('base dp1 ADAM_CHUNKED=$v', d['ms_per_step'], d['config'].get('dp_mode_select'), d['config']['last_loss'])"
done
done
