set -uo pipefail
O=gpurun_out/c21; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_graph.py tests/test_gpu_dp.py > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -1 $O/t.log
A="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5"
for i in 1 2 3; do
for v in 0 1; do
timeout -k 10 300 python -u scripts/ab_run.py train.step.FUSED_FP8_ADAM=$v -- $A > $O/f$v$i.log 2>&1 || { tail -30 $O/f$v$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/f$v$i.log') if l.startswith('{')][0];print('FUSED_FP8_ADAM=$v', d['ms_per_step'], d['config']['last_loss'])"
done
done
