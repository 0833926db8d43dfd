set -uo pipefail
O=gpurun_out/c28; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_fp8.py -k "test_gemm_fp8 or dgrad" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -3 $O/t.txt
timeout -k 10 300 python3 -u scripts/fp8_ring_lab.py > $O/lab.txt 2>&1; rc=$?; cat $O/lab.txt; exit $rc
