set -uo pipefail
O=gpurun_out/c48; mkdir -p $O
export TDG_NO_AUTOBUILD=1
timeout -k 10 600 python3 -u scripts/gemm_vs_blas.py --preset big --cfgs 0,4,9,10,12,13,20,21,22 > $O/big.txt 2>&1 || { tail -20 $O/big.txt; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/c48/big.txt'):
    if not l.startswith('{'): continue
    d=json.loads(l)
    if 'total_us' in d: print(d); continue
    print(f"{d['kind']:6s} {d['name']:6s} {d['M']}x{d['N']}x{d['K']} blas {d['blas_us']:7.1f}  best cfg{d['best']} {d['best_us']:7.1f}  ratio {d['best_us']/d['blas_us']:.2f}")
PY
