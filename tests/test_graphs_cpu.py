"""SegmentedGraph's item bookkeeping on CPU (train/graphs.py): host calls
recorded with cut() end a segment, calls recorded with pre() are replayed
just before the segment that was open when they were recorded and never cut
it, and abort() drops everything. The HIP graph itself is replaced by a
recorder (the GPU behaviour is tests/test_gpu_signal.py)."""
import contextlib

import pytest
import torch

from tensorflow_distributed_on_gke_amd.train import graphs


class _FakeGraph:
    n = 0

    def __init__(self):
        _FakeGraph.n += 1
        self.id = _FakeGraph.n
        self.log = None

    def capture_begin(self, pool=None, capture_error_mode=None):
        pass

    def capture_end(self):
        pass

    def replay(self):
        self.log.append(f"g{self.id}")


@pytest.fixture
def fake_cuda(monkeypatch):
    monkeypatch.setattr(torch.cuda, "CUDAGraph", _FakeGraph)
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    _FakeGraph.n = 0


def _bind(sg, log):
    for kind, x in sg.items:
        if kind == "graph":
            x.log = log


def test_pre_calls_replay_before_their_segment(fake_cuda):
    log = []
    sg = graphs.SegmentedGraph(stream=object(), pool=object())
    sg.begin()                                # segment g1
    sg.pre(lambda: log.append("issue-a"))
    sg.cut(lambda: log.append("wait-x"))      # g1 ends; g2 opens
    sg.pre(lambda: log.append("issue-b"))
    sg.pre(lambda: log.append("issue-c"))
    sg.cut(lambda: log.append("wait-y"))      # g2 ends; g3 opens
    sg.end()
    assert sg.num_graphs == 3 and sg.num_calls == 5
    assert [k for k, _ in sg.items] == ["call", "graph", "call", "call", "call", "graph", "call", "graph"]
    _bind(sg, log)
    sg.replay()
    assert log == ["issue-a", "g1", "wait-x", "issue-b", "issue-c", "g2", "wait-y", "g3"]


def test_pre_outside_capture_raises(fake_cuda):
    sg = graphs.SegmentedGraph(stream=object(), pool=object())
    with pytest.raises(RuntimeError):
        sg.pre(lambda: None)
    with pytest.raises(RuntimeError):
        sg.cut(lambda: None)


def test_abort_drops_pending_pre_calls(fake_cuda):
    log = []
    sg = graphs.SegmentedGraph(stream=object(), pool=object())
    sg.begin()
    sg.pre(lambda: log.append("stale"))
    sg.abort()
    assert sg.items == [] and not sg.capturing
    sg.begin()
    sg.end()
    _bind(sg, log)
    sg.replay()
    assert log == ["g2"]  # the aborted capture's pre call is gone
