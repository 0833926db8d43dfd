#!/usr/bin/env python3
"""Per-kernel L2 table from rocprofv3 --pmc passes (mean per dispatch):
TCC_HIT_sum, TCC_MISS_sum, the L2 hit rate HIT / (HIT + MISS) (the guide's
definition), TCC_EA0_RDREQ_sum (read requests L2 sent to the fabric:
Infinity Cache or HBM) and FETCH_SIZE (KiB) where collected. Sorted by
misses x dispatches.  usage: l2_table.py DIR [name-filter]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, filt=""):
    agg = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            n = r.get("Kernel_Name", "")
            if filt and filt not in n:
                continue
            agg[n[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))

    def m(cs, k):
        v = cs.get(k)
        return sum(v) / len(v) if v else float("nan")

    rows = []
    for n, cs in agg.items():
        cnt = max(len(v) for v in cs.values())
        mi = m(cs, "TCC_MISS_sum")
        rows.append(((mi if mi == mi else 0) * cnt, n, cs, cnt))
    print(f"# {d}\n{'calls':>6} {'hit_M':>8} {'miss_M':>8} {'hit%':>6} {'eaRdM':>8} {'fetchMB':>8}  kernel")
    for _, n, cs, cnt in sorted(rows, key=lambda r: -r[0]):
        h, mi = m(cs, "TCC_HIT_sum"), m(cs, "TCC_MISS_sum")
        hr = 100 * h / (h + mi) if (h + mi) == (h + mi) and (h + mi) > 0 else float("nan")
        print(f"{cnt:6d} {h / 1e6:8.3f} {mi / 1e6:8.3f} {hr:6.1f} {m(cs, 'TCC_EA0_RDREQ_sum') / 1e6:8.3f} "
              f"{m(cs, 'FETCH_SIZE') / 1024:8.1f}  {n}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
