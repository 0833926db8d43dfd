set -uo pipefail
O=gpurun_out/c35; mkdir -p $O
export TDG_NO_AUTOBUILD=1
TDG_ATTN_DQ3=1 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_fp8.py -k "attn or attention" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -1 $O/t.txt
for r in 1 2 3; do
  for v in 0 1; do
    echo "== DQ3=$v run $r"
    TDG_ATTN_DQ3=$v ATTN_B=16 ATTN_H=16 ATTN_L=512 timeout -k 10 120 python3 -u scripts/attn_bench.py 2>&1 | grep -v amdgpu.ids
  done
done
