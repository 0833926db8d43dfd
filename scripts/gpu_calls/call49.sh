set -uo pipefail
O=gpurun_out/c49; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 900 python3 -u scripts/tune_in_model.py --preset base --steps 20 --rounds 3 --out $O/tuned_base.json > $O/tune_base.log 2>&1 || { tail -20 $O/tune_base.log; exit 1; }
grep -v amdgpu.ids $O/tune_base.log | grep "start\|end\|was" | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['key'], d['was'], '->', d['best'], min(d['us_step'].values()))
    else: print(l.strip())"
python3 - <<'PY'
import json
cur=json.load(open('tensorflow_distributed_on_gke_amd/ops/gemm_tuned_gfx950.json'))
cur.update(json.load(open('gpurun_out/c49/tuned_base.json')))
json.dump(cur, open('gpurun_out/c49/table_new.json','w'), indent=0, sort_keys=True)
PY
run() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.log 2>&1 || { tail -30 $O/$n.log; exit 1; }; python -c "import json;d=[json.loads(l) for l in open('$O/$n.log') if l.startswith('{')][0];print('$n', d['ms_per_step'])"; }
for r in 1 2 3; do
  TDG_GEMM_TUNED_FILE=$O/table_new.json run new$r --steps 40 --warmup 10
  run old$r --steps 40 --warmup 10
done
