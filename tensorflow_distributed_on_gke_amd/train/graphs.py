"""A training step as a chain of HIP graphs cut at its host-issued collectives.

The data-parallel step cannot be one plain graph replay without putting the
RCCL collectives inside the capture (TDG_DP_GRAPH=full, see TrainStep), and
running it eagerly costs ~5-6 ms of host enqueue per step for ~5.5 ms of GPU
work (docs/ROADMAP.md item 5): each rank is launch-bound. The segmented graph
keeps the collectives as ordinary eager `torch.distributed` calls and captures
everything between them:

    graph 0 | all_reduce(span 0) | graph 1 | all_reduce(span 1) | ... |
    wait(span 0) | graph k (Adam of span 0) | wait(span 1) | ...

With the host comm thread (parallel/ddp.py) an issue point does not cut the
graph at all: a signal kernel captured at that point tells the thread when
the span is final, and the thread's job is handed over before the graph is
replayed (pre()). Only the waits remain as cuts.

While the step is captured, every point where the data-parallel code would
issue or wait for a collective ends the current graph and records the host
call instead; replay launches the graphs and the recorded calls in the same
order on the same stream. The collectives are the same RCCL calls the eager
step makes, so correctness across ranks does not depend on RCCL's own graph
support, and the per-step host cost drops to a few graph launches plus the
collective calls (one per all-reduce span).

Cuts can come from the autograd engine's device thread (gradient-ready hooks
fire inside backward), so captures use the "relaxed" mode: a capture begun
on one thread may be ended on another. All segments share one memory pool and
replay in capture order, so tensors that live across a cut keep their
addresses.
"""
from __future__ import annotations

import gc
import warnings
from typing import Callable, List, Optional, Tuple

import torch


class SegmentedGraph:
    def __init__(self, stream: Optional[torch.cuda.Stream] = None, pool=None):
        self.stream = stream
        # (a pool shared with other captured steps: train/step.py's shape cache)
        self.pool = pool
        self.items: List[Tuple[str, object]] = []
        self._cur: Optional[torch.cuda.CUDAGraph] = None
        # host calls to replay before the graph now being captured (pre())
        self._pre: List[Callable[[], None]] = []
        self.capturing = False

    # ------------------------------------------------------------------ capture
    def begin(self) -> None:
        """Start capturing on the current stream (must not be the default
        stream); the caller keeps that stream current until end()."""
        if self.stream is None:
            self.stream = torch.cuda.current_stream()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        self.capturing = True
        self._open()

    def _open(self) -> None:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(self.stream):
            g.capture_begin(pool=self.pool, capture_error_mode="relaxed")
        self._cur = g

    def _close(self) -> None:
        # two cuts back to back (e.g. a span's all-reduce issue followed by a
        # wait) leave an empty segment; replaying it costs ~1 us of host time
        with torch.cuda.stream(self.stream), warnings.catch_warnings():
            warnings.filterwarnings("ignore", message="The CUDA Graph is empty")
            self._cur.capture_end()
        self.items.extend(("call", fn) for fn in self._pre)
        self._pre = []
        self.items.append(("graph", self._cur))
        self._cur = None

    def cut(self, fn: Callable[[], None]) -> None:
        """End the running graph, record `fn` as a host call replayed between
        it and the next graph, and continue capturing."""
        if not self.capturing:
            raise RuntimeError("SegmentedGraph.cut outside a capture")
        self._close()
        self.items.append(("call", fn))
        self._open()

    def pre(self, fn: Callable[[], None]) -> None:
        """Record `fn` as a host call replayed just BEFORE the graph now being
        captured, without cutting it: for work the host hands off ahead of
        the GPU (a comm-thread job that waits for a signal kernel captured
        later in this same graph, parallel/ddp.py)."""
        if not self.capturing:
            raise RuntimeError("SegmentedGraph.pre outside a capture")
        self._pre.append(fn)

    def end(self) -> None:
        self._close()
        self.capturing = False

    def abort(self) -> None:
        """Drop a failed capture (ends the open stream capture if any)."""
        if self._cur is not None:
            try:
                with torch.cuda.stream(self.stream):
                    self._cur.capture_end()
            except Exception:  # pragma: no cover - best effort on an invalidated capture
                pass
            self._cur = None
        self.capturing = False
        self.items = []
        self._pre = []

    # ------------------------------------------------------------------ replay
    @property
    def num_graphs(self) -> int:
        return sum(1 for k, _ in self.items if k == "graph")

    @property
    def num_calls(self) -> int:
        return sum(1 for k, _ in self.items if k == "call")

    def replay(self) -> None:
        for kind, x in self.items:
            if kind == "graph":
                x.replay()
            else:
                x()


def prepare_capture() -> None:
    """What torch.cuda.graph does before a capture: idle device, no garbage
    whose frees could land inside the capture."""
    torch.cuda.synchronize()
    gc.collect()
    torch.cuda.empty_cache()
