set -uo pipefail
O=gpurun_out/c16; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 900 python3 -u scripts/tune_in_model.py --preset base --steps 20 --rounds 3 --out $O/tuned_base.json > $O/tune_base.log 2>&1 || { tail -20 $O/tune_base.log; exit 1; }
grep -v amdgpu.ids $O/tune_base.log | grep "start\|end\|was" | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(d['key'], d['was'], '->', d['best'], min(d['us_step'].values()))
    else: print(l.strip())"
python3 scripts/merge_tuned.py $O/tuned_base.json
run() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.log 2>&1 || { tail -30 $O/$n.log; exit 1; }; python -c "import json;d=[json.loads(l) for l in open('$O/$n.log') if l.startswith('{')][0];print('$n', d['ms_per_step'], d['value'], d['config']['last_loss'])"; }
run base1 && run base2 && run big1 --preset big --steps 20 --warmup 5 && run big2 --preset big --steps 20 --warmup 5 && \
run b8a --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 && \
run b16 --preset big --seq-len 512 --local-batch 16 --steps 20 --warmup 5
