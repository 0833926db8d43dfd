set -uo pipefail
O=gpurun_out/c6; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 python3 scripts/wgrad_fp8_one.py | tee $O/times.txt || exit 1
export REPS=3
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -- python3 scripts/wgrad_fp8_one.py > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/p2 -o p2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAVES -- python3 scripts/wgrad_fp8_one.py > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/p3 -o p3 --pmc FETCH_SIZE TCC_HIT_sum -- python3 scripts/wgrad_fp8_one.py > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
python3 scripts/pmc_summary.py $O wgrad_fp8 > $O/summary.txt
python3 scripts/pmc_summary.py $O gemm256 >> $O/summary.txt
cat $O/summary.txt
