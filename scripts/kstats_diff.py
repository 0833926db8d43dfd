#!/usr/bin/env python3
"""Per-kernel A/B of two rocprofv3 *_kernel_stats.csv files (same steps):
    python3 scripts/kstats_diff.py new.csv old.csv <steps>"""
import csv
import sys


def load(p):
    return {r["Name"]: (float(r["TotalDurationNs"]), int(r["Calls"])) for r in csv.DictReader(open(p))}


a, b, steps = load(sys.argv[1]), load(sys.argv[2]), float(sys.argv[3])
print(f"total new {sum(v[0] for v in a.values()) / 1e6 / steps:.3f} ms/step, "
      f"old {sum(v[0] for v in b.values()) / 1e6 / steps:.3f}")
rows = []
for k in set(a) | set(b):
    ta, ca = a.get(k, (0.0, 0))
    tb, cb = b.get(k, (0.0, 0))
    rows.append(((ta - tb) / 1e3 / steps, ta / 1e3 / steps, tb / 1e3 / steps, ca / steps, cb / steps, k))
print("  d_us/step   new_us    old_us  calls(new/old)  kernel")
for d, ta, tb, ca, cb, k in sorted(rows, key=lambda r: -abs(r[0]))[:25]:
    print(f"{d:10.1f} {ta:9.1f} {tb:9.1f}  {ca:5.1f}/{cb:5.1f}  {k[:100]}")
