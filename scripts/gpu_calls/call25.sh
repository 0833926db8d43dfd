set -uo pipefail
O=gpurun_out/c25; mkdir -p $O
export TDG_NO_AUTOBUILD=1
for i in 1 2 3; do
for v in 0 1; do
timeout -k 10 300 env TDG_DP_COMM_THREAD=$v python -u bench.py --force-dp 1 > $O/c$v$i.log 2>&1 || { tail -30 $O/c$v$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/c$v$i.log') if l.startswith('{')][0];print('dp1 COMM_THREAD=$v', d['ms_per_step'], d['config'].get('dp_mode_select'), d['config']['last_loss'])"
done
done
timeout -k 10 300 python -u bench.py > $O/single.log 2>&1 && python -c "import json;d=[json.loads(l) for l in open('$O/single.log') if l.startswith('{')][0];print('single graph', d['ms_per_step'])"
