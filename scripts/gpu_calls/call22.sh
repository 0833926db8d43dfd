set -uo pipefail
O=gpurun_out/c22; mkdir -p $O
export TDG_NO_AUTOBUILD=1
for i in 1 2 3; do
for v in 0 1; do
timeout -k 10 300 python -u scripts/ab_run.py train.optim.ADAM_CHUNKED=$v -- --preset big --steps 20 --warmup 5 > $O/b$v$i.log 2>&1 || { tail -30 $O/b$v$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/b$v$i.log') if l.startswith('{')][0];print('big ADAM_CHUNKED=$v', d['ms_per_step'], d['config']['last_loss'])"
done
done
for i in 1 2; do
for v in 0 1; do
timeout -k 10 300 python -u scripts/ab_run.py train.optim.ADAM_CHUNKED=$v -- > $O/s$v$i.log 2>&1 || { tail -30 $O/s$v$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/s$v$i.log') if l.startswith('{')][0];print('base ADAM_CHUNKED=$v', d['ms_per_step'], d['config']['last_loss'])"
done
done
