#!/usr/bin/env python3
"""Merge an in-model tuning result (scripts/tune_in_model.py --out) into the
in-tree GEMM table: python3 scripts/merge_tuned.py gpurun_out/.../tuned.json"""
import json
import os
import sys

T = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                 "tensorflow_distributed_on_gke_amd", "ops", "gemm_tuned_gfx950.json")
cur = json.load(open(T))
for path in sys.argv[1:]:
    for k, v in json.load(open(path)).items():
        if cur.get(k) != v:
            print(f"{k}: {cur.get(k)} -> {v}")
        cur[k] = v
json.dump(cur, open(T, "w"), indent=0, sort_keys=True)
