#!/usr/bin/env python3
"""One training step of a rocprofv3 --kernel-trace CSV in dispatch order:
kernel, grid (workgroups), duration and the gap before it, so every GEMM /
LayerNorm / attention launch can be told apart by position and shape.

    python3 scripts/ktrace_order.py <dir or kernel_trace.csv> [step index from the end, default 1]

Steps are delimited by the batch-prep kernel that opens every step."""
import csv
import glob
import os
import sys


def load(path):
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def short(name: str) -> str:
    name = name.replace("void ", "").replace("tdg::", "")
    cut = name.find("(")
    return name[:cut] if cut > 0 else name


def main(path, back=1):
    rows = load(path)
    starts = [i for i, r in enumerate(rows) if "prep_batch_kernel" in r["Kernel_Name"]]
    starts.append(len(rows))
    lo, hi = starts[-back - 1], starts[-back]
    sel = rows[lo:hi]
    t0 = int(sel[0]["Start_Timestamp"])
    prev_end = t0
    busy = 0
    print(f"{'#':>4} {'t_us':>8} {'gap':>6} {'dur_us':>7} {'grid':>7} {'wg':>5}  kernel")
    for i, r in enumerate(sel):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
        wg = int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0)
        nwg = grid // wg if wg else 0
        busy += e - s
        print(f"{i:4d} {(s - t0) / 1e3:8.1f} {(s - prev_end) / 1e3:6.1f} {(e - s) / 1e3:7.2f} "
              f"{nwg:7d} {wg:5d}  {short(r['Kernel_Name'])[:90]}")
        prev_end = e
    wall = int(sel[-1]["End_Timestamp"]) - t0
    print(f"# {len(sel)} dispatches, busy {busy / 1e6:.3f} ms, wall {wall / 1e6:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
