#!/usr/bin/env python3
"""Idle gaps between consecutive kernels of the last N training steps of a
rocprofv3 --kernel-trace CSV (steps delimited by the batch-prep kernel):
total idle time per step and the largest gaps with their neighbours."""
import csv
import glob
import os
import sys


def main(d, nsteps=5, top=12):
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(tr)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "prep_batch_kernel" in r["Kernel_Name"]]
    lo, hi = starts[-nsteps - 1], starts[-1]
    sel = rows[lo:hi]
    gaps = []
    end = int(sel[0]["End_Timestamp"])
    for a, b in zip(sel, sel[1:]):
        end = max(end, int(a["End_Timestamp"]))
        g = int(b["Start_Timestamp"]) - end
        if g > 0:
            gaps.append((g, a["Kernel_Name"][:60], b["Kernel_Name"][:60]))
    wall = int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])
    idle = sum(g for g, _, _ in gaps)
    print(f"# {tr}: last {nsteps} steps, wall {wall / 1e3 / nsteps:.1f} us/step, "
          f"idle {idle / 1e3 / nsteps:.1f} us/step in {len(gaps) / nsteps:.0f} gaps/step")
    agg = {}
    for g, a, b in gaps:
        k = (a, b)
        c = agg.setdefault(k, [0, 0])
        c[0] += 1
        c[1] += g
    for (a, b), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / 1e3 / nsteps:8.1f} us/step {c / nsteps:4.1f}x  {a}  ->  {b}")


if __name__ == "__main__":
    main(sys.argv[1], *(int(x) for x in sys.argv[2:]))
