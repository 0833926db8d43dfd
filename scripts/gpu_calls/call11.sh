set -uo pipefail
O=gpurun_out/c11; mkdir -p $O
export TDG_NO_AUTOBUILD=1
A="--preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 20 --warmup 5"
for i in 1 2 3; do
for v in 1 0; do
timeout -k 10 300 python -u scripts/ab_run.py ops.fp8.ATTN_BWD_G8=$v -- $A > $O/g8_${v}_$i.log 2>&1 || { tail -30 $O/g8_${v}_$i.log; exit 1; }
python -c "import json;d=[json.loads(l) for l in open('$O/g8_${v}_$i.log') if l.startswith('{')][0];print('ATTN_BWD_G8=$v', d['ms_per_step'], d['config']['last_loss'])"
done
done
