set -uo pipefail
O=gpurun_out/c3; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
prof() { local n=$1; shift; mkdir -p $O/prof_$n; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$n -o run -- python3 bench.py --steps 8 --warmup 3 --graph 0 "$@" > $O/prof_$n.log 2>&1 || { echo "prof $n failed"; tail -20 $O/prof_$n.log; exit 1; }; python3 scripts/prof_summary.py $O/prof_$n > $O/prof_$n/summary.txt; head -40 $O/prof_$n/summary.txt | cut -c1-150; }
prof big512_fp8 --preset big --seq-len 512 --local-batch 16 --dtype fp8
