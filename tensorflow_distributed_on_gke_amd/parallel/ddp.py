"""Synchronous data parallelism over RCCL (xGMI) with backward-overlapped,
ready-driven gradient all-reduce.

Replaces the reference's tf.distribute.MultiWorkerMirroredStrategy gradient
aggregation (reference: distributed_training_transformer/cluster/cluster.py:66,
__main__.py:105-132 -- loss scaled by 1/workers, SUM all-reduce inside
`apply_gradients`, initial variables broadcast from worker 0).

Design (MI355X): the model's gradients live in one flat f32 buffer laid out in
backward order (models/params.py), so gradients complete roughly front to
back. Every layer op notifies `grad_ready(param)` once it has written a
gradient; the DataParallel keeps the *frontier* -- the longest prefix of the
flat buffer whose gradients are all final -- and all-reduces the span between
the last reduced offset and the frontier:
  * as soon as the span reaches `bucket_mb` (the classic bucket), and
  * at every sync point (`ParamStore.grad_sync`, issued after each flush of
    the deferred weight-gradient GEMMs) once it is >= `min_mb`,
so collective boundaries follow the real completion order of the step instead
of a fixed bucket grid (a fixed grid straddling two flushes delays its
collective to the later one). On the GPU each span's all-reduce is issued by a
host thread (CommThread) on a communication stream once the compute stream has
reached the span's issue point, so communication overlaps the rest of backward
without the communication stream ever waiting on the compute stream on the
GPU (that handoff costs the compute stream ~55 us per span on MI355X); the
compute stream waits on the finished all-reduce device-side, and the host only
waits until the collective has been enqueued. In the segmented HIP graph the
issue point is a signal kernel inside the graph (ops/kernels.StreamSignal) the
thread spins on, so issuing costs no graph cut and no event record
(DP_SIGNAL; one-rank step 4.58 -> 4.54 ms, profiles/r6/dp_signal_issue.txt). Large spans (tens of MB) are what a
ring all-reduce over point-to-point xGMI needs to spread over RCCL's channels
and the 7 links per GPU.
"""
from __future__ import annotations

import math
import os
import queue
import sys
import threading
from dataclasses import dataclass
from typing import Callable, List, Optional

import torch
import torch.distributed as dist

from tensorflow_distributed_on_gke_amd.models.params import Param, ParamStore
from tensorflow_distributed_on_gke_amd.parallel.dist import PG_TIMEOUT_S


# Issue the gradient collectives from a host thread (CommThread) instead of
# making the communication stream wait on the compute stream.
#   "auto" (default): both issue paths are kept ready; TrainStep.choose_dp_mode
#          times them on the node the job runs on (segmented HIP graph and eager
#          step, each with the thread and with the process group's own stream
#          handoff), checks that the replicas stay bitwise equal after each
#          (verify_replicas) and keeps the faster verified one. Where no
#          start-up measurement runs (uncaptured step, autoselect off) the
#          thread is used: it won the one-rank RCCL A/B on MI355X (5.10-5.12 ms
#          vs 5.33-5.35 without, profiles/r4/ab_dp_comm_thread.txt). The
#          choice and its reason go into the bench record.
#   "1":   thread on RCCL (no measurement);  "0": never;
#   "force": thread also over gloo (GPU tensors: the multi-rank rehearsals on
#          one GPU, tests/test_gpu_dp.py; CPU tensors: tests/test_parallel_cpu.py).
COMM_THREAD = os.environ.get("TDG_DP_COMM_THREAD", "auto")
# tests: each thread-issued collective first sleeps a random 0..N ms (per-rank
# jitter in issue timing; replicas must stay bitwise equal and nothing hangs)
ISSUE_JITTER_MS = float(os.environ.get("TDG_DP_ISSUE_JITTER_MS", "0") or 0)
# seconds the host waits for the comm thread to enqueue a collective before
# the data-parallel state is poisoned and the step raises (a GPU that never
# reaches the issue point would otherwise hang); default: the process-group
# timeout (parallel/dist.py). A stall is reported every ISSUE_REPORT_S.
COMM_ISSUE_TIMEOUT_S = PG_TIMEOUT_S
ISSUE_REPORT_S = 60.0
# Segmented graph + comm thread: mark issue points with a signal kernel inside
# the graph (ops/kernels.StreamSignal) instead of cutting the graph and
# recording an event there ("0": the event cut).
DP_SIGNAL = os.environ.get("TDG_DP_SIGNAL", "1") != "0"


class CommThread:
    """Issues the data-parallel collectives from one host thread, each once the
    compute stream has passed its issue point (an event recorded there, or in
    a segmented graph the StreamSignal kernel captured there), on a
    communication stream that never waits on the compute stream on the GPU.

    Why: on MI355X a stream waiting on an event still pending on another
    stream costs the producing (compute) stream ~55 us per handoff -- 0.3 ms
    per step for the five all-reduce spans of Transformer-base -- while the
    reverse wait (compute waits for the finished all-reduce) and a plain event
    record are cheap (scripts/seg_comm_probe.py, docs/ROADMAP.md). One thread
    issues everything, so every rank issues its collectives in the same
    order, as ProcessGroupNCCL requires. CPU tensors (gloo rehearsals): no
    streams; the job issues the collective and waits for it on the thread."""

    def __init__(self, device: torch.device):
        self.device = device
        self.cuda = device.type == "cuda"
        self.stream = torch.cuda.Stream(device) if self.cuda else None
        self.signal = None
        if self.cuda and DP_SIGNAL:
            from tensorflow_distributed_on_gke_amd.ops.kernels import StreamSignal

            self.signal = StreamSignal(device)
        self._q: "queue.Queue[Optional[Callable[[], None]]]" = queue.Queue()
        self._t = threading.Thread(target=self._run, name="tdg-comm", daemon=True)
        self._t.start()

    def _run(self) -> None:
        if self.cuda:
            torch.cuda.set_device(self.device)
        while True:
            job = self._q.get()
            if job is None:
                return
            job()

    def submit(self, job: Callable[[], None]) -> None:
        self._q.put(job)

    def abandon(self) -> None:
        """Drop every queued job (after a failure the sequence is broken)."""
        try:
            while True:
                self._q.get_nowait()
        except queue.Empty:
            pass

    def close(self) -> bool:
        """Stop the thread; False if it did not exit (a job is stuck)."""
        if self._t.is_alive():
            self._q.put(None)
            self._t.join(timeout=60)
        return not self._t.is_alive()


class Pending:
    """Handle of an asynchronous collective issued through DataParallel.
    `work` is the process group's Work once the collective has been issued
    (at replay time when the step is a segmented graph, train/graphs.py).
    Thread-issued collectives also carry `issued` (set by the comm thread once
    the collective is enqueued), `done` (event on the comm stream after it)
    and `error`."""
    __slots__ = ("owner", "work", "issued", "done", "error")

    def __init__(self, owner: "DataParallel"):
        self.owner = owner
        self.work = None
        self.issued: Optional[threading.Event] = None
        self.done = None
        self.error: Optional[BaseException] = None

    def wait(self) -> None:
        """The current stream waits for the collective (device-side)."""
        self.owner._wait(self)


@dataclass
class Bucket:
    start: int
    end: int
    params: List[int]
    remaining: int = 0
    work: Optional[object] = None
    updated: bool = False


def plan_buckets(store: ParamStore, bucket_bytes: int) -> List[Bucket]:
    """The static bucket grid (cut at parameter boundaries into buckets of at
    least `bucket_bytes`, the last may be smaller): the spans the frontier
    launches when every gradient arrives one at a time in flat order. Pure."""
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
                 force: bool = False, min_mb: float = 4.0):
        self.store = store
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        # `force`: run the collective path with a single rank (tests the RCCL
        # plumbing on one GPU)
        self.active = self.world > 1 or (force and dist.is_initialized())
        self.overlap = overlap
        self.comm_dtype = comm_dtype
        self.bucket_elems = max(64, int(bucket_mb * 1024 * 1024) // 4)
        self.min_elems = max(64, int(min_mb * 1024 * 1024) // 4)
        self._order = sorted(store.params, key=lambda p: p.offset)
        self._pos = {p.index: i for i, p in enumerate(self._order)}
        self._comm_bufs = {}
        self.opt = None
        self._upd_stream = None
        # a train/graphs.SegmentedGraph while the step is being captured: the
        # collectives become host calls between graph segments
        self.recorder = None
        # collectives issued from a host thread (CommThread): `_comm` is the
        # thread when this configuration may use one, `_thread` the issue
        # path in use (None: the process group's own stream handoff)
        self._comm: Optional[CommThread] = None
        self._thread: Optional[CommThread] = None
        if self.active and COMM_THREAD != "0":
            nccl = store.flat.is_cuda and dist.get_backend(group) == "nccl"
            if nccl or COMM_THREAD == "force":
                self._comm = CommThread(store.flat.device)
                # (auto: on until TrainStep.choose_dp_mode measures otherwise)
                self._thread = self._comm
        # how the issue path was chosen (introspection / the bench record)
        self.comm_choice = "thread" if self._thread is not None else "pg"
        # collectives issued but not yet waited for (any issue path): a
        # main-thread collective issued meanwhile could interleave differently
        # on different ranks, so those check this is zero (check_quiescent)
        self._outstanding = 0
        # set (with the reason) once a collective failed or was not issued in
        # time: every later collective raises instead of risking a mismatched
        # sequence across ranks
        self.poisoned: Optional[str] = None
        self.buckets: List[Bucket] = []       # this step's launched spans
        self.last_buckets: List[Bucket] = []  # the previous step's (introspection)
        if self.active:
            store.on_grad_ready(self._on_ready)
            store.on_grad_sync(self._on_sync)
        self.reset()

    def attach_optimizer(self, opt, release: bool = True) -> None:
        """Run the optimizer per bucket (Adam over its flat range) instead of
        once after every all-reduce. finish() updates each bucket as soon as
        ITS all-reduce is done, so the Adam of the early buckets overlaps the
        all-reduce of the last one (the exposed tail). release=True also
        updates buckets mid-backward, once the model passed a release point
        (ParamStore.release_point: no later backward kernel reads those
        weights) -- the decoder side during the encoder's backward. The
        optimizer must offer apply_range(start, end, inc_step) / advance_step()."""
        if not self.active:
            return
        self.opt = opt
        if release:
            if self.store.flat.is_cuda:
                self._upd_stream = torch.cuda.Stream(self.store.flat.device)
            self.store.on_release(self._on_release)

    # ------------------------------------------------------------------ init
    def broadcast_params(self, src: int = 0) -> None:
        """Rank `src`'s initial weights to everyone (MWMS variable broadcast)."""
        if self.active:
            self.check_quiescent("broadcast_params")
            dist.broadcast(self.store.flat, src, group=self.group)
            self.store.refresh_compute()

    # ------------------------------------------------------------------ step
    def reset(self) -> None:
        if self.buckets:
            self.last_buckets = self.buckets
        self.buckets = []
        self._ready = [False] * len(self._order)
        self._front = 0      # params [0, _front) of the flat order are all final
        self._reduced = 0    # flat offset up to which all-reduces are launched

    def _front_off(self) -> int:
        if self._front >= len(self._order):
            return self.store.total
        return self._order[self._front].offset

    def _launch_span(self, end: int) -> None:
        if end <= self._reduced:
            return
        lo = self._reduced
        params = [p.index for p in self._order if lo <= p.offset < end]
        b = Bucket(lo, end, params)
        self._reduced = end
        self.buckets.append(b)
        self._launch(b)

    def _launch(self, b: Bucket) -> None:
        self._launch_now(b)

    def _launch_now(self, b: Bucket) -> None:
        view = self.store.flat_grad[b.start:b.end]
        if self.comm_dtype is not None and self.comm_dtype != view.dtype:
            buf = self._comm_bufs.get((b.start, b.end))
            if buf is None:
                buf = torch.empty(view.numel(), dtype=self.comm_dtype, device=view.device)
                self._comm_bufs[(b.start, b.end)] = buf
            buf.copy_(view)
            b.work = (self.all_reduce_async(buf), buf, view)
        else:
            b.work = (self.all_reduce_async(view), None, None)

    # ------------------------------------------------------------------ collectives
    def all_reduce_async(self, t: torch.Tensor) -> Pending:
        """SUM all-reduce of `t` in place, asynchronous. Under a segmented
        capture it is recorded as a host call between graph segments (so it
        is issued at replay, on the stream the graphs replay on)."""
        h = Pending(self)
        grp = self.group
        th = self._thread

        # under a segmented capture with the comm thread: no cut at the issue
        # point -- a signal kernel captured here tells the thread when the
        # span is final, and the job is handed over before the graph replays
        sig = (th.signal if th is not None and self.recorder is not None else None)

        def issue():
            self._check_poison()
            self._outstanding += 1
            if th is None:
                h.work = dist.all_reduce(t, group=grp, async_op=True)
                return
            cuda = th.cuda
            ready = expect = None
            if sig is not None:
                sig.expected += 1
                expect = sig.expected
            elif cuda:
                ready = torch.cuda.Event()
                ready.record()  # the current (compute) stream: t is final here
            h.issued = threading.Event()
            h.error = None
            jitter = ISSUE_JITTER_MS

            def job():
                try:
                    if jitter > 0:
                        import random
                        import time
                        time.sleep(random.uniform(0.0, jitter) / 1e3)
                    if cuda:
                        if sig is not None:
                            if not sig.wait(expect, COMM_ISSUE_TIMEOUT_S):
                                raise RuntimeError(f"stream signal {expect} not reached within "
                                                   f"{COMM_ISSUE_TIMEOUT_S:.0f} s (at {sig.value()})")
                        else:
                            ready.synchronize()
                        with torch.cuda.stream(th.stream):
                            w = dist.all_reduce(t, group=grp, async_op=True)
                            w.wait()  # comm stream after the collective
                            done = torch.cuda.Event()
                            done.record(th.stream)
                    else:  # CPU (gloo): complete before `issued` is set
                        w = dist.all_reduce(t, group=grp, async_op=True)
                        w.wait()
                        done = None
                    h.work, h.done = w, done
                except BaseException as e:  # surfaced by the waiter
                    h.error = e
                finally:
                    h.issued.set()

            th.submit(job)

        if sig is not None:
            sig.emit()  # captured at the issue point
            self.recorder.pre(issue)
        elif self.recorder is not None:
            self.recorder.cut(issue)
        else:
            issue()
        return h

    def _check_poison(self) -> None:
        if self.poisoned is not None:
            raise RuntimeError(f"data-parallel state is poisoned ({self.poisoned}); refusing further "
                               "collectives -- exit and restart the job")

    def _poison(self, reason: str) -> None:
        self.poisoned = reason
        if self._comm is not None:
            # a stuck job keeps later ones queued behind it: drop them all
            self._comm.abandon()

    def check_quiescent(self, what: str) -> None:
        """Every collective this object issued has been waited for: `what` (a
        main-thread collective) cannot interleave with them differently on
        different ranks. Raises otherwise, and when poisoned."""
        self._check_poison()
        if self._outstanding:
            raise RuntimeError(f"{what}: {self._outstanding} data-parallel collective(s) issued but not "
                               "waited for (call finish() first)")

    @property
    def can_thread(self) -> bool:
        """A comm thread exists, so the issue path can be switched."""
        return self._comm is not None

    def use_thread(self, on: bool) -> None:
        """Select the issue path for collectives issued from now on (a
        segmented graph captured earlier keeps the path it was captured
        with). Only between steps: nothing may be in flight."""
        self.check_quiescent("use_thread")
        if on and self._comm is None:
            raise RuntimeError("no comm thread in this configuration (TDG_DP_COMM_THREAD)")
        self._thread = self._comm if on else None
        self.comm_choice = "thread" if on else "pg"

    def _wait_now(self, h: Pending) -> None:
        """Current stream waits for the collective (device-side; the host only
        waits until a thread-issued collective has been enqueued)."""
        self._check_poison()
        if h.issued is None:
            h.work.wait()
            self._outstanding -= 1
            return
        waited = 0.0
        while not h.issued.wait(timeout=min(ISSUE_REPORT_S, COMM_ISSUE_TIMEOUT_S - waited)):
            waited += ISSUE_REPORT_S
            if waited >= COMM_ISSUE_TIMEOUT_S:
                msg = (f"collective not issued within {COMM_ISSUE_TIMEOUT_S:.0f} s (the compute stream "
                       "never reached its issue point)")
                self._poison(msg)
                raise RuntimeError("data-parallel " + msg)
            print(f"[rank {self.rank}] data-parallel: waiting {waited:.0f} s for a collective to be "
                  "issued", file=sys.stderr, flush=True)
        if h.error is not None:
            self._poison(f"collective failed on the comm thread: {h.error!r}")
            raise RuntimeError("data-parallel collective failed on the comm thread") from h.error
        if h.done is not None:
            torch.cuda.current_stream().wait_event(h.done)
        self._outstanding -= 1

    def _wait(self, h: Pending) -> None:
        if self.recorder is not None:
            self.recorder.cut(lambda: self._wait_now(h))
        else:
            self._wait_now(h)

    def _on_ready(self, p: Param) -> None:
        self._ready[self._pos[p.index]] = True
        while self._front < len(self._order) and self._ready[self._front]:
            self._front += 1
        if self.overlap and self._front_off() - self._reduced >= self.bucket_elems:
            self._launch_span(self._front_off())

    def _on_sync(self) -> None:
        if self.overlap and self._front_off() - self._reduced >= self.min_elems:
            self._launch_span(self._front_off())

    def _complete(self, b: Bucket) -> None:
        """Current stream waits for the bucket's all-reduce (device-side)."""
        self._complete_many([b])

    def _complete_many(self, bs: List[Bucket]) -> None:
        hs = [b.work[0] for b in bs]
        if self.recorder is not None:  # one host call between two graph segments
            self.recorder.cut(lambda: [self._wait_now(h) for h in hs])
        else:
            for h in hs:
                h.wait()
        for b in bs:
            _, buf, view = b.work
            if buf is not None:
                view.copy_(buf)

    def _on_release(self) -> None:
        if self.opt is None:
            return
        ready = [b for b in self.buckets if b.work is not None and not b.updated]
        if not ready:
            return
        if self._upd_stream is None:  # CPU (gloo): in order
            for b in ready:
                self._complete(b)
                self.opt.apply_range(b.start, b.end, inc_step=False)
                b.updated = True
            return
        upd = self._upd_stream
        # ordered after every kernel issued so far (the last reads of these weights)
        upd.wait_stream(torch.cuda.current_stream(upd.device))
        with torch.cuda.stream(upd):
            for b in ready:
                self._complete(b)
                self.opt.apply_range(b.start, b.end, inc_step=False)
                b.updated = True

    def finish(self) -> None:
        """Launch the rest of the buffer and make the current stream wait for
        every collective (device-side wait; no host sync). With an attached
        optimizer, also update every span not yet updated and advance the
        optimizer step."""
        if not self.active:
            self.reset()
            return
        self._launch_span(self.store.total)
        if self._upd_stream is not None:
            torch.cuda.current_stream(self._upd_stream.device).wait_stream(self._upd_stream)
        # Work.wait() orders the current stream after the collective. Two
        # groups, so a segmented graph keeps two wait points: the spans
        # launched well before the end of backward (normally complete by now)
        # and the last two -- the one launched at the last layer end, just
        # before backward finishes, and the one launched just above. The Adam
        # of the first group runs while those two all-reduces are in flight
        # (and while the host thread issues them: the first wait does not
        # block the host on a span issued moments ago).
        todo = [b for b in self.buckets if not b.updated]
        cut = -2 if len(todo) >= 3 else -1
        for grp in (todo[:cut], todo[cut:]):
            if not grp:
                continue
            self._complete_many(grp)
            if self.opt is not None:
                for b in grp:
                    self.opt.apply_range(b.start, b.end, inc_step=False)
        if self.opt is not None:
            self.opt.advance_step()
        self.reset()

    def verify_replicas(self) -> None:
        """Debug check (race / divergence detection): every rank's weights must
        be bitwise identical after a synchronous step. Compares an exact
        checksum (sum of the int32 bit patterns, int64) across ranks."""
        if self.world <= 1:
            return
        self.check_quiescent("verify_replicas")
        bits = self.store.flat.detach().view(torch.int32)
        local = torch.stack([bits.sum(dtype=torch.int64), (bits.to(torch.int64) * 2654435761).sum()])
        allv = [torch.zeros_like(local) for _ in range(self.world)]
        dist.all_gather(allv, local, group=self.group)
        ref = allv[0]
        bad = [r for r, v in enumerate(allv) if not torch.equal(v, ref)]
        if bad:
            raise RuntimeError(f"replica divergence: ranks {bad} differ from rank 0 "
                               f"({[tuple(v.tolist()) for v in allv]})")

    def close(self) -> None:
        """Stop the comm thread (all its collectives have been waited for).
        Raises if it is stuck, so the process exits non-zero instead of
        tearing the process group down under a collective."""
        if self._comm is not None:
            ok = self._comm.close()
            self._comm = self._thread = None
            if not ok:
                raise RuntimeError("data-parallel comm thread did not stop (a collective is stuck)")

    def allreduce_metrics(self, t: torch.Tensor) -> torch.Tensor:
        if self.world > 1:
            self.check_quiescent("allreduce_metrics")
            dist.all_reduce(t, group=self.group)
        return t

    def barrier(self) -> None:
        if self.world > 1:
            self.check_quiescent("barrier")
            from tensorflow_distributed_on_gke_amd.parallel import dist as tdist
            tdist.barrier()
