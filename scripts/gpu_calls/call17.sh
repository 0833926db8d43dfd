set -uo pipefail
O=gpurun_out/c17; mkdir -p $O
export TDG_NO_AUTOBUILD=1
export -f true 2>/dev/null; run() { n=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$n.log 2>&1 || { tail -30 $O/$n.log; exit 1; }; python -c "import json;d=[json.loads(l) for l in open('$O/$n.log') if l.startswith('{')][0];print('$n', d['ms_per_step'], d['config']['last_loss'])"; }
for i in 1 2 3; do
TDG_GEMM_TUNED_FILE=ab_old/old_table.json run base_old$i || exit 1
run base_new$i || exit 1
done
for i in 1 2; do
TDG_GEMM_TUNED_FILE=ab_old/old_table.json run big_old$i --preset big --steps 20 --warmup 5 || exit 1
run big_new$i --preset big --steps 20 --warmup 5 || exit 1
done
