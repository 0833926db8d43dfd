"""Cost of a graph-segment boundary on the compute stream (what the segmented
data-parallel step adds per cut): one graph of 2n kernels against two graphs
of n replayed back to back, with and without an event record / cross-stream
wait / host callback between them. Prints us per boundary."""
import sys
import time

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda")
x = torch.randn(8192, 1024, device=dev, dtype=torch.bfloat16)
w = torch.randn(1024, 1024, device=dev, dtype=torch.bfloat16)
side = torch.cuda.Stream()
cap = torch.cuda.Stream()


def work(k):
    y = x
    for _ in range(k):
        y = torch.mm(y, w) * 0.01
    return y


def graph(k):
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.stream(cap):
        work(k)  # warm
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=cap):
        work(k)
    return g


one = graph(2 * n)
a, b = graph(n), graph(n)
ev = torch.cuda.Event()


def run(kind, iters=50):
    with torch.cuda.stream(cap):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(iters):
                if kind == "one":
                    one.replay()
                    continue
                a.replay()
                if kind in ("event", "event+wait"):
                    ev.record()
                if kind == "event+wait":
                    side.wait_event(ev)
                if kind == "event+sync":
                    ev.record()
                    ev.synchronize()
                b.replay()
            torch.cuda.synchronize()
            t = (time.perf_counter() - t0) / iters * 1e6
    return t


base = run("one")
print(f"one graph of {2*n} GEMM+scale pairs: {base:.1f} us")
for kind in ("two", "event", "event+wait", "event+sync"):
    t = run(kind)
    print(f"{kind:>11}: {t:.1f} us  (+{t - base:.1f} us per boundary)")
