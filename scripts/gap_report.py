"""Idle gaps inside one training step of a rocprofv3 kernel trace: steps are
delimited by the per-step batch-prep kernel; prints each step's dispatch count,
span and busy time, and the gaps above a threshold in the second-to-last step.
usage: gap_report.py <kernel_trace.csv> [min_gap_us=3]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
thr = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "prep_batch_kernel" in r["Kernel_Name"]]
for a, b in zip(idx[-6:-1], idx[-5:]):
    seg = rows[a:b]
    t0, t1 = int(seg[0]["Start_Timestamp"]), int(rows[b]["Start_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    print(f"step: {len(seg)} dispatches, span {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us")
a, b = idx[-3], idx[-2]
prev = None
tot = 0.0
for i in range(a, b + 1):
    r = rows[i]
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if prev is not None and s - prev > thr * 1e3:
        tot += (s - prev) / 1e3
        print(f"{i - a:4d} gap {(s - prev) / 1e3:6.1f} us before {r['Kernel_Name'][:70]}"
              f"  (after {rows[i - 1]['Kernel_Name'][:50]})")
    prev = max(prev or 0, e)
print(f"gaps > {thr} us: {tot:.1f} us")
