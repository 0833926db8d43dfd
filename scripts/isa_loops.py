#!/usr/bin/env python3
"""Compress a kernel's gfx950 assembly to its schedule skeleton: labels,
branches, waits, barriers, LDS-DMA issues, with runs of MFMAs / LDS reads
collapsed to counts. Shows whether the compiler kept a hand-placed phase
schedule (e.g. MFMAs sunk out of their phases into the loop latch).

    hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S -o k.s kernel.hip
    python3 scripts/isa_loops.py k.s <kernel-name-substring> [first-line [last-line]]
"""
import re
import sys


def main():
    path, name = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and name in l)
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    body = lines[st:en]
    lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    hi = int(sys.argv[4]) if len(sys.argv) > 4 else len(body)
    run, kind = 0, None

    def flush():
        nonlocal run, kind
        if run:
            print(f"      [{run} x {kind}]")
        run, kind = 0, None

    for i, l in enumerate(body[lo:hi], lo):
        t = l.strip()
        if not t or t.startswith(";") or (t.startswith(".") and not t.startswith(".LBB")):
            continue
        op = t.split()[0]
        k = None
        if op.startswith("v_mfma"):
            k = "mfma"
        elif op.startswith("ds_read") or op.startswith("ds_load"):
            k = "ds_read"
        elif op.startswith("ds_write") or op.startswith("ds_store"):
            k = "ds_write"
        elif op.startswith("v_"):
            k = "valu"
        elif op.startswith("s_") and not (op.startswith("s_waitcnt") or op.startswith("s_barrier")
                                          or op.startswith("s_cbranch") or op.startswith("s_branch")
                                          or op.startswith("s_setprio")):
            k = "salu"
        if k is not None:
            if k != kind:
                flush()
                kind = k
            run += 1
            continue
        flush()
        print(f"{i:6d}  {t[:90]}")
    flush()


if __name__ == "__main__":
    main()
