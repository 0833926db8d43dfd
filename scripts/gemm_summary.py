#!/usr/bin/env python3
import json, sys
for r in json.load(open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gemm_bench.json")):
    cf = {k: v for k, v in r.items() if k.startswith("cfg")}
    top = sorted(cf.items(), key=lambda kv: kv[1])[:3]
    print(f"{r['name']:12s} blt {r['hipblaslt_us']:7.2f}us  best {r['best_us']:7.2f}us {r['best_tflops']:6.1f}TF  {top}  err {r['rel_err']}")
