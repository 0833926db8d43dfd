set -uo pipefail
O=gpurun_out/c26; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
for cfg in "base:" "big:--preset big" "fp8:--preset big --seq-len 512 --local-batch 16 --dtype fp8"; do
n=${cfg%%:*}; a=${cfg#*:}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o p -- python3 bench.py $a --steps 10 --warmup 3 --graph 0 > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
f=$(find $O/$n -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" 13 > $O/$n.txt; head -16 $O/$n.txt
done
