set -uo pipefail
O=gpurun_out/c18; mkdir -p $O
export TDG_NO_AUTOBUILD=1 ATTN_B=16 ATTN_H=16 ATTN_L=512
timeout -k 10 200 python3 -u scripts/attn_bench.py > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
grep -v amdgpu $O/bench.txt
bash scripts/pmc_attn.sh c18/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cat gpurun_out/c18/pmc/summary.txt
