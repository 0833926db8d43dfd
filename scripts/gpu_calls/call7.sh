set -uo pipefail
O=gpurun_out/c7; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 240 env TDG_PKG_ROOT=ab_old python3 -u scripts/fp8_ab_lab.py > $O/old.txt 2>&1 || { tail -5 $O/old.txt; exit 1; }
timeout -k 10 240 python3 -u scripts/fp8_ab_lab.py > $O/new.txt 2>&1 || { tail -5 $O/new.txt; exit 1; }
cat $O/old.txt $O/new.txt
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py > $O/tests.txt 2>&1; r=$?; tail -5 $O/tests.txt; exit $r
