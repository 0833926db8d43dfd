set -uo pipefail
O=gpurun_out/c9; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/pytest.log | head -80; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py > $O/base_$i.log 2>&1 || { tail -30 $O/base_$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/base_$i.log') if l.startswith('{')][0];print('base', d['ms_per_step'], d['value'], d['config']['last_loss'])"
done
timeout -k 10 300 python -u bench.py --preset big --steps 20 --warmup 5 > $O/big.log 2>&1 || { tail -30 $O/big.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/big.log') if l.startswith('{')][0];print('big', d['ms_per_step'], d['config']['last_loss'])"
timeout -k 10 300 python -u bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5 > $O/b8.log 2>&1 || { tail -30 $O/b8.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/b8.log') if l.startswith('{')][0];print('big512 fp8', d['ms_per_step'], d['config']['last_loss'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pbase -o p -- python3 bench.py --steps 10 --warmup 3 --graph 0 > $O/pbase.log 2>&1 || { tail -20 $O/pbase.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p8 -o p -- python3 bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 10 --warmup 3 --graph 0 > $O/p8.log 2>&1 || { tail -20 $O/p8.log; exit 1; }
for d in pbase p8; do f=$(find $O/$d -name "*kernel_stats.csv" | head -1); echo "== $d $f"; python3 scripts/kstats.py "$f" 13 > $O/$d.txt; head -30 $O/$d.txt; done
