#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel time over the LAST
N training steps only (steps delimited by the batch-prep kernel that opens
every step -- the Adam kernel when it is absent; the data-parallel path runs
one Adam per bucket -- so autotuning and warm-up dispatches are excluded), as
ms per step."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, nsteps=5):
    traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    rows = list(csv.DictReader(open(traces[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    ends = [i - 1 for i, r in enumerate(rows) if "prep_batch_kernel" in r["Kernel_Name"]]
    if len(ends) > nsteps:
        ends.append(len(rows) - 1)  # the last step runs to the end of the trace
    else:
        ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    if len(ends) > nsteps:
        lo, hi = ends[-nsteps - 1] + 1, ends[-1] + 1
    else:
        lo, hi = 0, len(rows)
    sel = rows[lo:hi]
    n = max(1, min(nsteps, len(ends) - 1))
    agg = defaultdict(lambda: [0, 0.0])
    for r in sel:
        name = r["Kernel_Name"]
        agg[name][0] += 1
        agg[name][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in agg.values())
    wall = int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])
    print(f"# {traces[0]}\n# last {n} steps: kernel busy {tot/1e6/n:.3f} ms/step, "
          f"wall {wall/1e6/n:.3f} ms/step, {len(sel)//n} dispatches/step")
    print(f"{'pct':>6} {'ms/step':>8} {'calls/st':>8} {'avg_us':>8}  kernel")
    for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{100*t/tot:6.2f} {t/1e6/n:8.3f} {c/n:8.1f} {t/c/1e3:8.2f}  {name[:100]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 5)
