#!/bin/bash
# Full-size data-parallel rehearsal on ONE MI355X (no scaling curve: eight
# ranks share the card and talk over gloo): Transformer-base, the real 64 MB
# bucket plan over the 221 MB gradient buffer, the measured issue-path / mode
# selection (choose_dp_mode, its start-up seconds recorded) and bitwise replica
# verification after the timed steps. Then the one-rank RCCL data-parallel
# step (--force-dp 1) against the single graph, interleaved.
set -uo pipefail
TAG=${1:-r6dp}
O=gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
( while sleep 45; do echo "[tick] $(date +%T)"; done ) &
TICK=$!
trap "kill $TICK 2>/dev/null" EXIT
echo "== 8 gloo ranks, Transformer-base"
# one hardware queue per rank: eight processes x the default 4 queues
# oversubscribe the card's queue slots (the first attempt of this rehearsal
# died with an illegal-instruction abort inside a PyTorch kernel)
GPU_MAX_HW_QUEUES=1 TDG_DIST_BACKEND=gloo timeout -k 10 900 python -u bench.py --gpus 8 --steps 6 --warmup 2 --verify-replicas 1 \
  > $O/dp8.log 2>&1
rc=$?
grep -E "dp_mode_select|^\{" $O/dp8.log | cut -c1-900
[ $rc -eq 0 ] || { tail -40 $O/dp8.log; exit $rc; }
echo "== one rank: RCCL data-parallel step vs single graph"
for r in 1 2 3; do
  for v in 0 1; do
    timeout -k 10 300 python -u bench.py --force-dp $v > $O/f${v}_$r.log 2>&1 || { tail -20 $O/f${v}_$r.log; exit 1; }
    echo "force_dp=$v run=$r $(grep '^{' $O/f${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"].get("dp_mode_select"), d["config"].get("comm_issue"))')"
  done
done
