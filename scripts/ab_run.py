#!/usr/bin/env python3
"""Run bench.py in-process with module attributes overridden (A/B of
switches that are module constants):
    python3 scripts/ab_run.py ops.fp8.ATTN_BWD_G8=0 -- --preset big --seq-len 512 ...
"""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("TDG_PKG_ROOT"):  # another copy of the package (and its built _C)
    sys.path.insert(0, os.path.abspath(os.environ["TDG_PKG_ROOT"]))
import tensorflow_distributed_on_gke_amd  # noqa: E402,F401  (cached: bench.py gets this copy)
print(f"[ab_run] package {os.path.dirname(tensorflow_distributed_on_gke_amd.__file__)}", file=sys.stderr)
i = sys.argv.index("--")
for a in sys.argv[1:i]:
    name, val = a.split("=", 1)
    mod, attr = name.rsplit(".", 1)
    m = importlib.import_module("tensorflow_distributed_on_gke_amd." + mod)
    old = getattr(m, attr)
    if isinstance(old, tuple):
        setattr(m, attr, tuple(int(x) for x in val.split(",")))
    else:
        setattr(m, attr, type(old)(int(val)) if isinstance(old, (bool, int)) else type(old)(val))
    print(f"[ab_run] {name} = {getattr(m, attr)!r}", file=sys.stderr)
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[i + 1:]
runpy.run_path(sys.argv[0], run_name="__main__")
