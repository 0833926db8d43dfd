"""Weight-gradient side stream.

Backward has one critical path: the activation-gradient chain (LayerNorm
backward -> dgrad GEMM -> attention backward -> dgrad ...). Weight-gradient
GEMMs and bias column sums hang off it: nothing later in backward reads
them. They are issued on a second HIP stream, forked from the compute stream
at the point their inputs exist, so they fill the CUs the dgrad chain leaves
idle (small GEMM tails, LayerNorm, attention). The gradient all-reduce of a
bucket is launched from the side stream after it has caught up with the
compute stream (parallel/ddp.py), and the optimizer joins both streams.

Inside a HIP-graph capture the fork/join become graph edges, so the replayed
step keeps the concurrency. Off by default (`TDG_SIDE_STREAM=1` enables it):
measured on MI355X at Transformer-base / batch 64 it did not pay (8.34 vs
8.13 ms/step) -- the GEMMs already fill the chip and the two streams contend.
"""
from __future__ import annotations

import os
from contextlib import contextmanager
from typing import Dict, Optional

import torch

ENABLED = os.environ.get("TDG_SIDE_STREAM", "0") != "0"
_SIDE: Dict[int, torch.cuda.Stream] = {}


def side(device: torch.device) -> Optional[torch.cuda.Stream]:
    if not ENABLED or device.type != "cuda":
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _SIDE.get(idx)
    if s is None:
        with torch.cuda.device(idx):
            s = torch.cuda.Stream()
        _SIDE[idx] = s
    return s


@contextmanager
def offload(*tensors: torch.Tensor):
    """Run the enclosed kernels on the side stream, ordered after everything
    already queued on the current stream; `tensors` (inputs the side kernels
    read) are kept alive for the side stream."""
    dev = tensors[0].device
    s = side(dev)
    if s is None:
        yield
        return
    main = torch.cuda.current_stream(dev)
    s.wait_stream(main)
    with torch.cuda.stream(s):
        yield
    for t in tensors:
        t.record_stream(s)


def join(device: torch.device) -> None:
    """Make the current stream wait for all side-stream work."""
    s = side(device)
    if s is not None:
        torch.cuda.current_stream(device).wait_stream(s)


@contextmanager
def on_side(device: torch.device):
    """Enter the side stream after it caught up with the current stream (for
    collectives that consume gradients produced on both streams)."""
    s = side(device)
    if s is None:
        yield
        return
    s.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(s):
        yield
