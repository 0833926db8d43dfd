set -uo pipefail
O=gpurun_out/c20; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attn or attention" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for i in 1 2; do
timeout -k 10 200 env TDG_PKG_ROOT=ab_old python3 -u scripts/attn_bench.py 2>&1 | grep -v amdgpu | sed 's/^/old /'
timeout -k 10 200 python3 -u scripts/attn_bench.py 2>&1 | grep -v amdgpu | sed 's/^/new /'
done
for i in 1 2 3; do
for v in old new; do
if [ $v = old ]; then export TDG_PKG_ROOT=ab_old; else unset TDG_PKG_ROOT; fi
timeout -k 10 300 python -u scripts/ab_run.py -- > $O/$v$i.log 2>&1 || { tail -30 $O/$v$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/$v$i.log') if l.startswith('{')][0];print('base step $v', d['ms_per_step'], d['config']['last_loss'])"
done
done
