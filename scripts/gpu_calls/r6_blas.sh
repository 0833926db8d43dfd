#!/bin/bash
# In-tree GEMMs vs hipBLASLt on the Transformer-big (config 4) and -base
# shapes, (SCHEDS: labels of repeated runs).
#   bash scripts/gpu_calls/r6_blas.sh TAG "SCHED_A SCHED_B"
set -uo pipefail
TAG=${1:-r6blas}; SCHEDS=${2:-"cur"}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
for p in big base; do
  for s in $SCHEDS; do
    TDG_G256_SCHED=$s timeout -k 10 300 python -u scripts/gemm_vs_blas.py --preset $p --cfgs 0,4,9,10,12,13,20,21,22 \
      > $O/vs_${p}_$s.jsonl 2>&1 || { tail -20 $O/vs_${p}_$s.jsonl; exit 1; }
    python3 - $O/vs_${p}_$s.jsonl $p $s <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
for r in rows:
    if "name" in r:
        print(f"{sys.argv[2]} sched={sys.argv[3]} {r['kind']:5s} {r['name']:6s} {r['M']}x{r['N']}x{r['K']} blas {r['blas_us']:7.1f} best cfg{r['best']:<2d} {r['best_us']:7.1f} ratio {r['best_us']/r['blas_us']:.2f}  " + " ".join(f"c{c}={r.get('cfg'+str(c),'-')}" for c in (12, 20, 21, 22, 9, 10)))
    else:
        print(sys.argv[2], "sched", sys.argv[3], r)
PY
  done
done
