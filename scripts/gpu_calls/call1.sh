set -uo pipefail
mkdir -p gpurun_out/c1
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 700 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_fp8.py tests/test_gpu_dp.py tests/test_gpu_kernels.py -k "fp8 or wgrad_ragged or gemm256" > gpurun_out/c1/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/c1/pytest.log | tail -80 > gpurun_out/c1/pytest_summary.txt
tail -5 gpurun_out/c1/pytest_summary.txt
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/c1/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python -u scripts/wgrad_lab.py > gpurun_out/c1/wgrad_lab.txt 2>&1; rc=$?
cat gpurun_out/c1/wgrad_lab.txt | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/fp8_w1_lab.py > gpurun_out/c1/fp8_lab.txt 2>&1; rc=$?
cat gpurun_out/c1/fp8_lab.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/gemm_vs_blas.py --preset big --cfgs 0,12,13,14,20,21,22,23,24,25,26 > gpurun_out/c1/vs_blas_big.txt 2>&1; rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/c1/vs_blas_big.txt"):
    if l.startswith("{"):
        d = json.loads(l)
        if "name" in d:
            cf = " ".join(f"{k[3:]}:{v}" for k, v in d.items() if k.startswith("cfg"))
            print(d["kind"], d["name"], "blas", d["blas_us"], "best", d["best"], d["best_us"], "|", cf)
        else:
            print(d)
PY
exit $rc
