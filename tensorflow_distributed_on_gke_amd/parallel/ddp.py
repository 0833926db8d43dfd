"""Synchronous data parallelism over RCCL (xGMI) with bucketed, backward-
overlapped gradient all-reduce.

Replaces the reference's tf.distribute.MultiWorkerMirroredStrategy gradient
aggregation (reference: distributed_training_transformer/cluster/cluster.py:66,
__main__.py:105-132 — loss scaled by 1/workers, SUM all-reduce inside
`apply_gradients`, initial variables broadcast from worker 0).

Design (MI355X): the model's gradients live in one flat f32 buffer laid out in
backward order (models/params.py). The buffer is cut into contiguous buckets
of ~`bucket_mb`; each layer op notifies `grad_ready(param)` as soon as it has
written a gradient, and the bucket whose last gradient just landed is
all-reduced immediately with `async_op=True`. ProcessGroupNCCL (RCCL on ROCm)
runs the collective on its own HIP stream, ordered after the producing kernels
by an event, so communication overlaps the rest of backward; the optimizer's
stream waits on the outstanding work handles (no host sync). Buckets are large
(default 64 MB) because a ring all-reduce over point-to-point xGMI needs big
messages to spread over RCCL's channels / the 7 links per GPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist

from tensorflow_distributed_on_gke_amd.models.params import Param, ParamStore
from tensorflow_distributed_on_gke_amd.ops.streams import join, on_side


@dataclass
class Bucket:
    start: int
    end: int
    params: List[int]
    remaining: int = 0
    work: Optional[object] = None


def plan_buckets(store: ParamStore, bucket_bytes: int) -> List[Bucket]:
    """Cut the flat buffer (ordered by offset) at parameter boundaries into
    buckets of at least `bucket_bytes` (the last may be smaller). Pure."""
    order = sorted(store.params, key=lambda p: p.offset)
    buckets: List[Bucket] = []
    cur: Optional[Bucket] = None
    for p in order:
        end = p.offset + math.ceil(p.numel / 64) * 64
        if cur is None:
            cur = Bucket(p.offset, end, [p.index])
        else:
            cur.end = end
            cur.params.append(p.index)
        if (cur.end - cur.start) * 4 >= bucket_bytes:
            buckets.append(cur)
            cur = None
    if cur is not None:
        buckets.append(cur)
    if buckets:
        buckets[-1].end = store.total
    return buckets


class DataParallel:
    def __init__(self, store: ParamStore, bucket_mb: float = 64.0, group=None,
                 comm_dtype: Optional[torch.dtype] = None, overlap: bool = True,
                 force: bool = False):
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # `force`: run the collective path with a single rank (tests the RCCL
        # plumbing on one GPU)
        self.active = self.world > 1 or (force and dist.is_initialized())
        self.overlap = overlap
        self.comm_dtype = comm_dtype
        self.buckets = plan_buckets(store, int(bucket_mb * 1024 * 1024))
        self.bucket_of = {}
        for i, b in enumerate(self.buckets):
            for pi in b.params:
                self.bucket_of[pi] = i
        self._comm_bufs = {}
        if self.active:
            store.on_grad_ready(self._on_ready)
        self.reset()

    # ------------------------------------------------------------------ init
    def broadcast_params(self, src: int = 0) -> None:
        """Rank `src`'s initial weights to everyone (MWMS variable broadcast)."""
        if self.active:
            dist.broadcast(self.store.flat, src, group=self.group)
            self.store.refresh_compute()

    # ------------------------------------------------------------------ step
    def reset(self) -> None:
        for b in self.buckets:
            b.remaining = len(b.params)
            b.work = None

    def _launch(self, b: Bucket) -> None:
        # gradients come from both the compute stream and the weight-gradient
        # side stream: collect on the side stream after it caught up
        with on_side(self.store.flat_grad.device):
            self._launch_now(b)

    def _launch_now(self, b: Bucket) -> None:
        view = self.store.flat_grad[b.start:b.end]
        if self.comm_dtype is not None and self.comm_dtype != view.dtype:
            buf = self._comm_bufs.get(b.start)
            if buf is None:
                buf = torch.empty(view.numel(), dtype=self.comm_dtype, device=view.device)
                self._comm_bufs[b.start] = buf
            buf.copy_(view)
            b.work = (dist.all_reduce(buf, group=self.group, async_op=True), buf, view)
        else:
            b.work = (dist.all_reduce(view, group=self.group, async_op=True), None, None)

    def _on_ready(self, p: Param) -> None:
        b = self.buckets[self.bucket_of[p.index]]
        b.remaining -= 1
        if b.remaining == 0 and self.overlap and b.work is None:
            self._launch(b)

    def finish(self) -> None:
        """Launch any bucket not yet reduced and make the current stream wait
        for all of them (device-side wait; no host sync)."""
        join(self.store.flat_grad.device)
        if not self.active:
            self.reset()
            return
        for b in self.buckets:
            if b.work is None:
                self._launch(b)
        for b in self.buckets:
            work, buf, view = b.work
            work.wait()
            if buf is not None:
                view.copy_(buf)
        self.reset()

    def verify_replicas(self) -> None:
        """Debug check (race / divergence detection): every rank's weights must
        be bitwise identical after a synchronous step. Compares an exact
        checksum (sum of the int32 bit patterns, int64) across ranks."""
        if self.world <= 1:
            return
        bits = self.store.flat.detach().view(torch.int32)
        local = torch.stack([bits.sum(dtype=torch.int64), (bits.to(torch.int64) * 2654435761).sum()])
        allv = [torch.zeros_like(local) for _ in range(self.world)]
        dist.all_gather(allv, local, group=self.group)
        ref = allv[0]
        bad = [r for r, v in enumerate(allv) if not torch.equal(v, ref)]
        if bad:
            raise RuntimeError(f"replica divergence: ranks {bad} differ from rank 0 "
                               f"({[tuple(v.tolist()) for v in allv]})")

    def allreduce_metrics(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            dist.all_reduce(t, group=self.group)
        return t
