#!/bin/bash
# The one-rank data-parallel step (--force-dp 1: segmented graph, RCCL on one
# rank, measured issue-path selection) against the single graph, interleaved;
# then in-tree vs hipBLASLt on the Transformer-big GEMM shapes.
set -uo pipefail
O=gpurun_out/r6dpb
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 300 python -u bench.py --force-dp $v --steps 60 --warmup 15 > $O/dp${v}_$r.log 2>&1 || { tail -20 $O/dp${v}_$r.log; exit 1; }
    echo "[force-dp $v] run=$r $(grep '^{' $O/dp${v}_$r.log | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])') ms/step"
  done
done
grep -h "choose_dp_mode\|dp mode\|selected" $O/dp1_*.log | head -6
timeout -k 10 300 python -u scripts/gemm_vs_blas.py --preset big --cfgs 0,4,9,10,12,13,20,21,22 > $O/vs_big.jsonl 2>&1 || { tail -20 $O/vs_big.jsonl; exit 1; }
python3 - $O/vs_big.jsonl <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
for r in rows:
    if "name" in r:
        print(f"{r['kind']:5s} {r['name']:6s} {r['M']}x{r['N']}x{r['K']} blas {r['blas_us']:7.1f} best cfg{r['best']:<2d} {r['best_us']:7.1f} ratio {r['best_us']/r['blas_us']:.2f}")
    else:
        print(r)
PY
