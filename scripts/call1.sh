set -uo pipefail
mkdir -p gpurun_out/c1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_dp.py -k fp8 > gpurun_out/c1/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/c1/pytest.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/wgrad_lab.py > gpurun_out/c1/wgrad_lab.txt 2>&1; rc=$?
cat gpurun_out/c1/wgrad_lab.txt | tail -30
exit $rc
