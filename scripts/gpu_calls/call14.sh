set -uo pipefail
O=gpurun_out/c14; mkdir -p $O
export TDG_NO_AUTOBUILD=1
A="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5"
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
for v in old new; do
if [ $v = old ]; then export TDG_PKG_ROOT=ab_old; else unset TDG_PKG_ROOT; fi
timeout -k 10 300 python -u scripts/ab_run.py -- $A > $O/$v$i.log 2>&1 || { tail -30 $O/$v$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/$v$i.log') if l.startswith('{')][0];print('$v', d['ms_per_step'], d['config']['last_loss'])"
done
done
unset TDG_PKG_ROOT
timeout -k 10 240 env TDG_PKG_ROOT=ab_old python3 -u scripts/fp8_ab_lab.py > $O/lab_old.txt 2>&1 && timeout -k 10 240 python3 -u scripts/fp8_ab_lab.py > $O/lab_new.txt 2>&1; cat $O/lab_old.txt $O/lab_new.txt | grep -v amdgpu.ids
