#!/bin/bash
# Kernel trace of scripts/embed_csr_lab.py (CSR vs fixed-point embedding backward).
set -uo pipefail
O=gpurun_out/csrlab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
export TDG_NO_AUTOBUILD=1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o t -- python3 scripts/embed_csr_lab.py > $O/lab.log 2>&1 || { tail -20 $O/lab.log; exit 1; }
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
names = [r for r in rows if "embed" in r["Kernel_Name"]]
# 6 configs x (20 csr calls x 3 kernels + 20 fx calls x 2 kernels) = 100 dispatches each
per = 100
for c in range(len(names) // per):
    chunk = names[c * per:(c + 1) * per]
    d = collections.defaultdict(list)
    for r in chunk:
        d[r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0)
    print(c, "  ".join(f"{k.split('::')[-1]}={sorted(v)[len(v)//2]:.2f}" for k, v in d.items()))
PY
