"""The stream-position signal (csrc/kernels/signal.hip, ops/kernels.StreamSignal)
the data-parallel comm thread follows instead of a graph cut + event at each
all-reduce issue point, and SegmentedGraph.pre (host calls handed over before
a graph segment without cutting it)."""
import threading
import time

import pytest
import torch

from tensorflow_distributed_on_gke_amd.ops import kernels as kk

pytestmark = pytest.mark.gpu


def test_signal_follows_stream_order():
    s = kk.StreamSignal(torch.device("cuda", 0))
    assert s.value() == 0
    torch.cuda._sleep(200_000_000)  # ~0.1 s of GPU spin ahead of the signal
    s.emit()
    assert s.value() == 0, "signal published before the work queued ahead of it finished"
    assert s.wait(1, 30.0)
    assert s.value() == 1
    s.emit()
    s.emit()
    assert s.wait(3, 30.0)
    assert not s.wait(4, 0.05)  # never emitted: times out
    torch.cuda.synchronize()


def test_signal_inside_graph_replays():
    s = kk.StreamSignal(torch.device("cuda", 0))
    x = torch.randn(1024, 1024, device="cuda")
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        y = x @ x
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        y = x @ x
        s.emit()
        y = y @ x
        s.emit()
    assert s.value() == 0  # capture runs nothing
    for _ in range(3):
        g.replay()
    assert s.wait(6, 30.0)
    torch.cuda.synchronize()
    assert s.value() == 6


def test_signal_wakes_waiting_thread():
    """A host thread spinning in wait() (GIL released) while the main thread
    keeps running Python sees the signal."""
    s = kk.StreamSignal(torch.device("cuda", 0))
    seen = {}

    def waiter():
        t0 = time.perf_counter()
        seen["ok"] = s.wait(1, 30.0)
        seen["dt"] = time.perf_counter() - t0

    th = threading.Thread(target=waiter)
    th.start()
    n = 0
    for _ in range(20000):  # the GIL stays usable while the thread waits
        n += 1
    torch.cuda._sleep(50_000_000)
    s.emit()
    th.join(timeout=60)
    assert not th.is_alive() and seen["ok"] and n == 20000


def test_segmented_graph_pre_does_not_cut():
    from tensorflow_distributed_on_gke_amd.train.graphs import SegmentedGraph, prepare_capture

    x = torch.randn(256, 256, device="cuda")
    log = []
    st = torch.cuda.Stream()
    prepare_capture()
    sg = SegmentedGraph(stream=st)
    with torch.cuda.stream(st):
        sg.begin()
        y = x @ x
        sg.pre(lambda: log.append("pre1"))
        y = y @ x
        sg.cut(lambda: log.append("cut"))
        y = y @ x
        sg.pre(lambda: log.append("pre2"))
        sg.end()
    assert sg.num_graphs == 2 and sg.num_calls == 3
    kinds = [k for k, _ in sg.items]
    assert kinds == ["call", "graph", "call", "call", "graph"]
    sg.replay()
    torch.cuda.synchronize()
    assert log == ["pre1", "cut", "pre2"]
