set -uo pipefail
O=gpurun_out/c13; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p8 -o p -- python3 bench.py --preset big --seq-len 512 --local-batch 16 --dtype fp8 --steps 10 --warmup 3 --graph 0 > $O/p8.log 2>&1 || { tail -20 $O/p8.log; exit 1; }
f=$(find $O/p8 -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" 13 > $O/p8.txt; head -40 $O/p8.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pbig -o p -- python3 bench.py --preset big --steps 10 --warmup 3 --graph 0 > $O/pbig.log 2>&1 || { tail -20 $O/pbig.log; exit 1; }
f=$(find $O/pbig -name "*kernel_stats.csv" | head -1); python3 scripts/kstats.py "$f" 13 > $O/pbig.txt; head -30 $O/pbig.txt
