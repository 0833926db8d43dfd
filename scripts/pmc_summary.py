#!/usr/bin/env python3
"""Average PMC counter values per kernel from rocprofv3 --pmc csv output."""
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        n = r.get("Kernel_Name", "")
        if filt not in n:
            continue
        agg[n[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, cs in agg.items():
    print(n)
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
