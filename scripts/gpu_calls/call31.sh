set -uo pipefail
O=gpurun_out/c31; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fp8.py -k "test_gemm_fp8 or dgrad" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for r in 1 2; do
  unset TDG_PKG_ROOT; timeout -k 10 300 python3 -u scripts/fp8_ring_lab.py > $O/new$r.txt 2>&1 || { cat $O/new$r.txt; exit 1; }
  export TDG_PKG_ROOT=ab_old; timeout -k 10 300 python3 -u scripts/fp8_ring_lab.py > $O/old$r.txt 2>&1 || { cat $O/old$r.txt; exit 1; }
  echo "== new $r"; grep -v amdgpu.ids $O/new$r.txt; echo "== old $r"; grep -v amdgpu.ids $O/old$r.txt
done
