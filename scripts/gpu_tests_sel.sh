#!/bin/bash
# One GPU call: selected GPU tests (args: pytest selection), time-limited.
set -uo pipefail
O=gpurun_out/${TAG:-sel}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest -x -v --timeout 240 --timeout-method thread "$@" > $O/pytest.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" $O/pytest.log | tail -40
exit $rc
