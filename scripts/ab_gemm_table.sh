#!/bin/bash
# A/B of the GEMM tuning table: the tree's table vs an older copy ($1), the
# same kernels, interleaved runs on one box. Output: gpurun_out/ab_table.txt
set -o pipefail
OLD=$1
OUT=gpurun_out/ab_table.txt
: > $OUT
for preset in base big; do
  for r in 1 2; do
    for t in new old; do
      if [ $t = old ]; then export TDG_GEMM_TUNED_FILE=$OLD; else unset TDG_GEMM_TUNED_FILE; fi
      echo -n "$preset $t " >> $OUT
      timeout -k 10 240 python bench.py --preset $preset --steps 20 --warmup 5 2>/dev/null | tail -1 >> $OUT || exit 1
    done
  done
done
