#!/bin/bash
# Kernel-level profile of the headline bench on one MI355X:
#   rocprofv3 --kernel-trace --stats (no PMC counters in the same run)
# Writes under gpurun_out/prof_<tag>/ ; summarise with scripts/prof_summary.py
set -euo pipefail
TAG=${1:-base}
shift || true
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
  python3 bench.py --steps 10 --warmup 3 --graph 0 "$@" > "$OUT/bench.log" 2>&1
python3 scripts/prof_summary.py "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt" | head -60
