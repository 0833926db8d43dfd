#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: per-kernel total
time, calls, average, and share of GPU time."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d):
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        rows = list(csv.DictReader(open(stats[0])))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        print(f"# {stats[0]}\n# total kernel time {tot/1e6:.3f} ms")
        print(f"{'pct':>6} {'total_ms':>9} {'calls':>6} {'avg_us':>8}  kernel")
        for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:45]:
            t = float(r["TotalDurationNs"])
            print(f"{100*t/tot:6.2f} {t/1e6:9.3f} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:8.2f}  {r['Name'][:110]}")
        return
    traces = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    agg = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(traces[0])):
        n = r["Kernel_Name"]
        agg[n][0] += 1
        agg[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    tot = sum(v[1] for v in agg.values())
    for n, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:45]:
        print(f"{100*t/tot:6.2f} {t/1e6:9.3f} {c:6d} {t/c/1e3:8.2f}  {n[:110]}")


if __name__ == "__main__":
    main(sys.argv[1])
