#!/bin/bash
# A/B of the tuned-table change against ab_old/, then the big-preset re-tune.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
echo "== A/B headline"
bash scripts/ab_trees.sh $PWD/ab_old $PWD 3 || exit 1
echo "== big re-tune"
bash scripts/gpu_calls/r6_tune.sh big 4,9,10,12,13,20,22 > /dev/null 2>&1
rc=$?
grep -v "^{" gpurun_out/tune/big.log | tail -3
grep '"was"' gpurun_out/tune/big.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l)
    if d['was']!=d['best']: print(d['key'], d['was'], '->', d['best'], d['us_step'])
"
exit $rc
