set -uo pipefail
O=gpurun_out/c8; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 > $O/b8_$i.log 2>&1 || { tail -30 $O/b8_$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/b8_$i.log') if l.startswith('{')][0];print('big512 fp8', d['ms_per_step'], d['config']['last_loss'])"
done
timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --steps 20 --warmup 5 > $O/b16.log 2>&1 || { tail -30 $O/b16.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/b16.log') if l.startswith('{')][0];print('big512 bf16', d['ms_per_step'], d['config']['last_loss'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o p -- python3 bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 10 --warmup 3 --graph 0 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
tot=sum(float(r['TotalDurationNs']) for r in rows)
print('total ms per step (13 steps)', tot/1e6/13)
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6/13:8.3f} ms/step {int(r['Calls'])//13:5d}/step  {r['Name'][:110]}")
PY
