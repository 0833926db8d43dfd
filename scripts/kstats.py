#!/usr/bin/env python3
"""Per-step kernel table from a rocprofv3 *_kernel_stats.csv:
    python3 scripts/kstats.py <kernel_stats.csv> <steps profiled>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"# {sys.argv[1]}")
print(f"# kernel busy {tot / 1e6 / steps:.3f} ms/step, {calls / steps:.0f} dispatches/step (incl. warmup/setup averaged)")
print("   pct  ms/step calls/st   avg_us  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    t = float(r["TotalDurationNs"])
    print(f"{100 * t / tot:6.2f} {t / 1e6 / steps:8.3f} {int(r['Calls']) / steps:8.1f} "
          f"{t / 1e3 / int(r['Calls']):8.2f}  {r['Name'][:110]}")
