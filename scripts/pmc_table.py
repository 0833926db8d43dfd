#!/usr/bin/env python3
"""Per-kernel PMC table from the passes of scripts/pmc_bench.sh (mean per
dispatch over all dispatches of a kernel):
  wait%     SQ_WAIT_ANY / SQ_WAVE_CYCLES   share of wave time stalled
  mfma      SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES (relative MFMA activity:
            the two counters sum over different units, so this is a ratio
            between kernels, not a utilisation percentage)
  fetchMB   FETCH_SIZE / 1024              bytes fetched from L2/memory
  ldsconf%  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra LDS cycles)
  mfma/lds  SQ_INSTS_MFMA / SQ_INSTS_LDS
Sorted by fetched bytes x dispatches."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[r.get("Kernel_Name", "")[:80]][r["Counter_Name"]].append(float(r["Counter_Value"]))

    def m(cs, k):
        v = cs.get(k)
        return sum(v) / len(v) if v else float("nan")

    def ratio(a, b):
        return a / b if b and b == b else float("nan")

    rows = []
    for n, cs in agg.items():
        cnt = max(len(v) for v in cs.values())
        rows.append((m(cs, "FETCH_SIZE") * cnt, n, cs))
    print(f"# {d}\n{'wait%':>6} {'mfma':>6} {'fetchMB':>8} {'ldsconf%':>8} {'mfma/lds':>8}  kernel")
    for _, n, cs in sorted(rows, key=lambda r: -(r[0] if r[0] == r[0] else 0)):
        wait = 100 * ratio(m(cs, "SQ_WAIT_ANY"), m(cs, "SQ_WAVE_CYCLES"))
        mf = ratio(m(cs, "SQ_VALU_MFMA_BUSY_CYCLES"), m(cs, "SQ_BUSY_CYCLES"))
        conf = 100 * ratio(m(cs, "SQ_LDS_BANK_CONFLICT"), m(cs, "SQ_LDS_IDX_ACTIVE"))
        ml = ratio(m(cs, "SQ_INSTS_MFMA"), m(cs, "SQ_INSTS_LDS"))
        print(f"{wait:6.1f} {mf:6.2f} {m(cs, 'FETCH_SIZE') / 1024:8.1f} {conf:8.1f} {ml:8.2f}  {n}")


if __name__ == "__main__":
    main(sys.argv[1])
