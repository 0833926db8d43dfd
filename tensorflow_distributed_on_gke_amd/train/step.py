"""One synchronous data-parallel training step, optionally captured into a HIP
graph.

step = dropout-stream advance -> teacher-forced forward -> fused CE/accuracy ->
backward (gradients into the flat buffer, bucketed RCCL all-reduce started
from inside backward) -> wait for the buckets -> multi-tensor Adam.

Reference: distributed_training_transformer/__main__.py:105-132 (train_step
inside strategy.run, apply_gradients all-reduce, strategy.reduce(SUM) of the
per-replica losses). The per-step loss stays on device; it is summed over
replicas only when the host reads it (log points).
"""
from __future__ import annotations

import os
import time
from collections import OrderedDict
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from tensorflow_distributed_on_gke_amd.models.layers import RunCtx, WgradQueue
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer
from tensorflow_distributed_on_gke_amd.parallel import ddp as _ddp_mod
from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel
from tensorflow_distributed_on_gke_amd.ops import kernels as K
from tensorflow_distributed_on_gke_amd.train.graphs import SegmentedGraph, prepare_capture
from tensorflow_distributed_on_gke_amd.train.optim import Adam


# data parallel: weight gradients flushed in wave-sized chunks at layer ends
CHUNKED_WGRAD = True
# tiles per wave of the chunked schedule (0: one whole-K 256x256 tile per CU);
# tests set small values to force problems to be cut across launches
WAVE_TILES = 0
# skip the optimizer's gradient zeroing (all GPU gradient writers overwrite)
ZERO_GRAD_FREE = True
# how a data-parallel step is captured (TrainStep.capture):
#   "seg"  -- chain of HIP graphs cut at the collectives, which stay eager
#             RCCL calls between the segments (train/graphs.py; default)
#   "0"    -- no capture: the data-parallel step runs eagerly
# (round 1 also had "full", the collectives captured inside one graph; it
# failed capture under PyTorch 2.10's process-group watchdog and was removed)
DP_GRAPH = os.environ.get("TDG_DP_GRAPH", "seg")
# data parallel: time the segmented graph against the eager step once and keep
# the faster (TrainStep.choose_dp_mode); False keeps the segmented graph
DP_AUTOSELECT = True
# data parallel: each bucket's Adam runs as soon as its all-reduce is done.
# "tail": at the end of the step, so the last bucket's all-reduce overlaps the
# Adam of the others. "1": also mid-backward (decoder side during the
# encoder's backward) -- on one MI355X with --force-dp that concurrent Adam
# contended with the encoder backward for more than it hid (6.45 vs 6.34 ms).
# "0": one Adam after finish.
DP_OVERLAP_OPT = "tail"
# fp8 (one optimizer pass over the whole buffer): the Adam kernel also
# refreshes the e4m3 weight copies (no separate re-quantisation pass)
FUSED_FP8_ADAM = True


class TrainStep:
    def __init__(self, model: Transformer, opt: Adam, ddp: Optional[DataParallel], workers: float,
                 seed: int = 0, dropout: Optional[float] = None, fp8_state=None,
                 defer_wgrad: Optional[bool] = None, loss_mode: str = "replica_mean"):
        self.model = model
        self.opt = opt
        self.ddp = ddp
        self.workers = float(workers)
        # global token mean: every replica's loss is normalised by the label
        # count of the whole global batch (one scalar all-reduce per step,
        # overlapped with the forward) and the gradients are SUM-reduced
        if loss_mode not in ("replica_mean", "global_mean"):
            raise ValueError(f"loss_mode must be replica_mean or global_mean, got {loss_mode!r}")
        self.global_mean = loss_mode == "global_mean" and ddp is not None and ddp.world > 1
        self._ntok_sum = None
        if self.global_mean:
            self.workers = 1.0
            self._ntok_sum = ddp.all_reduce_async
        dev = model.device
        self.rt = RunCtx(training=True, dropout=model.cfg.dropout if dropout is None else dropout,
                         seed=seed, ctr=torch.zeros(1, dtype=torch.int64, device=dev),
                         store=model.store, fp8=fp8_state)
        # weight gradients grouped per shape (layers.WgradQueue): at the end of
        # backward on one GPU; with data parallelism also at the decoder /
        # encoder boundary so the decoder-side buckets' all-reduce overlaps
        # the encoder backward
        if defer_wgrad is None:
            defer_wgrad = True
        if defer_wgrad and dev.type == "cuda":
            dp = ddp is not None and ddp.active
            self.rt.wgrad = WgradQueue(flush_at_boundary=dp,
                                       wave_tiles=(WAVE_TILES or K.NUM_CU) if dp and CHUNKED_WGRAD else 0)
            # every encoder and decoder layer's backward ends with a layer_end()
            self.rt.wgrad.layers_per_step = 2 * model.cfg.layers
            # fp8: the bf16 weight gradients left (the vocab projection) are
            # too few tiles for the ragged 256x256 launch
            self.rt.wgrad.small_per_shape = fp8_state is not None and not self.rt.wgrad._chunking()
        self.fp8 = fp8_state
        if dev.type == "cuda" and not self.rt.accumulate and ZERO_GRAD_FREE:
            opt.zero_grad = False  # every GPU gradient writer overwrites
        mode = DP_OVERLAP_OPT
        # (fp8: the scale update and the e4m3 weight re-quantisation run after
        # ddp.finish(), when every bucket's Adam is done, so the per-bucket
        # Adam stays on; the mid-backward variant would update weights the
        # fp8 copies of which the encoder backward still reads)
        if ddp is not None and ddp.active and mode != "0" and not (fp8_state is not None and mode != "tail"):
            ddp.attach_optimizer(opt, release=mode != "tail")
        # metric accumulators [sum loss, sum acc, n steps, n tokens] (device)
        self.accum = torch.zeros(4, dtype=torch.float32, device=dev)
        self.last = torch.zeros(2, dtype=torch.float32, device=dev)
        self.graph = None
        self.segments: Optional[SegmentedGraph] = None
        self._static: Optional[Tuple[torch.Tensor, torch.Tensor]] = None
        # Variable-length batches (text data, the reference's padded-to-the-
        # batch-max shapes: english_portugese_dataset.py:44-46, __main__.py:127
        # experimental_relax_shapes): with `bucketed` set, a batch of a shape
        # not captured yet is captured on the spot (warm-up, restore, capture:
        # it still trains once) and kept in an LRU cache of at most
        # `graph_cache` captured steps keyed by (source, target) shape. All of
        # them allocate from ONE memory pool: each replay is a whole step, so
        # the intermediates of different shapes may share memory (workspaces,
        # which persist, are never reused: ops.kernels.workspace).
        self.bucketed = False
        self.graph_cache = 64
        self._graphs: "OrderedDict[tuple, tuple]" = OrderedDict()
        self._key: Optional[tuple] = None
        self._pool = None
        self._cap_stream: Optional[torch.cuda.Stream] = None
        self._warm_stream: Optional[torch.cuda.Stream] = None
        self.graph_stats = {"captures": 0, "replays": 0, "evictions": 0}

    @property
    def captured(self) -> bool:
        return self.graph is not None or self.segments is not None

    def capture_mode(self) -> str:
        """"single" (one graph, no collectives), "seg" or "0" (the
        data-parallel step stays eager)."""
        if self.ddp is None or not self.ddp.active:
            return "single"
        if DP_GRAPH not in ("seg", "0"):
            raise ValueError(f"TDG_DP_GRAPH must be seg or 0, got {DP_GRAPH!r}")
        if self.ddp._upd_stream is not None:
            # mid-backward Adam on its own stream would leave unjoined work
            # at a cut
            return "0"
        return DP_GRAPH

    # ------------------------------------------------------------------ state
    def _state(self):
        """Every tensor a training step mutates that outlives the step."""
        ts = [self.model.store.flat, self.opt.m, self.opt.v, self.opt.step, self.rt.ctr,
              self.accum, self.last]
        if self.fp8 is not None:
            ts += [self.fp8.meta.scale, self.fp8.gmeta.scale]
        return ts

    def snapshot(self):
        st = [t.clone() for t in self._state()]
        if self.fp8 is not None:
            st += [self.fp8.meta.amax.clone(), self.fp8.gmeta.amax.clone()]
        return st

    def restore(self, st) -> None:
        """Put back a snapshot(): weights (and their derived bf16 / transposed /
        fp8 copies), Adam moments and step, dropout counter, metric
        accumulators, fp8 scales."""
        for t, v in zip(self._state(), st):
            t.copy_(v)
        self.model.store.refresh_compute()
        if self.fp8 is not None:
            self.fp8.weights.refresh()  # e4m3 copies with the restored scales
            self.fp8.meta.amax.copy_(st[-2])
            self.fp8.gmeta.amax.copy_(st[-1])

    def eager(self, src: torch.Tensor, tgt: torch.Tensor) -> torch.Tensor:
        self.model.loss_and_backward(src, tgt, self.rt, self.workers, accum=self.accum,
                                     step_out=self.last, bump_ctr=True, ntok_sum=self._ntok_sum)
        if self.ddp is not None:
            self.ddp.finish()
        if self.ddp is None or self.ddp.opt is None:
            if self.fp8 is not None and FUSED_FP8_ADAM and \
                    self.fp8.weights.adam_chunks(self.model.store) is not None:
                # new scales, then Adam refreshing the e4m3 weight copies
                self.fp8.before_fused_opt()
                self.opt.apply(fp8w=self.fp8.weights)
                return self.last
            self.opt.apply()
        if self.fp8 is not None:
            self.fp8.after_step()  # new scales, then fp8 weight copies
        return self.last

    # ------------------------------------------------------------------ HIP graph
    def capture(self, src: torch.Tensor, tgt: torch.Tensor, warmup: int = 2) -> bool:
        """Capture the whole step (fwd+bwd+optimizer) on static input buffers:
        one HIP graph on a single GPU; under data parallelism a segmented
        graph whose collectives are eager calls between the segments.

        Warm-up steps run first (lazily-allocated workspaces, GEMM tunings,
        communication buffers); the training state is snapshotted before and
        restored after them, so capture() itself trains nothing: after it the
        model, optimizer and counters are exactly as they were. Returns False
        (and leaves the step eager) when the data-parallel step is configured
        not to be captured."""
        mode = self.capture_mode()
        if mode == "0":
            return False
        if self._pool is None:
            self._pool = torch.cuda.graph_pool_handle()
        if (self._static is not None and self._static[0].shape == src.shape
                and self._static[1].shape == tgt.shape):
            # (choose_dp_mode captures more than one arm: every captured graph
            # reads the same static input buffers)
            self._static[0].copy_(src)
            self._static[1].copy_(tgt)
        else:
            self._static = (src.clone(), tgt.clone())
        saved = self.snapshot()
        if self._cap_stream is None:
            # one warm-up and one capture stream for every captured shape: the
            # workspaces (keyed by stream) are shared by all of them
            self._warm_stream = torch.cuda.Stream()
            self._cap_stream = torch.cuda.Stream()
        s = self._warm_stream
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.eager(*self._static)
        torch.cuda.current_stream().wait_stream(s)
        self.restore(saved)
        del saved
        if mode != "single":
            # no collective of the warm-up may still be pending in the process
            # group's watchdog when the capture starts
            torch.cuda.synchronize()
            self.ddp.check_quiescent("capture")
            dist.barrier(group=self.ddp.group)
            torch.cuda.synchronize()
        if mode == "seg":
            prepare_capture()
            cap = self._cap_stream
            cap.wait_stream(torch.cuda.current_stream())
            rec = SegmentedGraph(cap, pool=self._pool)
            self.ddp.recorder = rec
            try:
                with torch.cuda.stream(cap):
                    rec.begin()
                    self.eager(*self._static)
                    rec.end()
            except BaseException:
                rec.abort()
                raise
            finally:
                self.ddp.recorder = None
            torch.cuda.current_stream().wait_stream(cap)
            self.segments = rec
            self._register()
            return True
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=self._pool, stream=self._cap_stream):
            self.eager(*self._static)
        self.graph = g
        self._register()
        return True

    # ------------------------------------------------------------------ shape cache
    def _register(self) -> None:
        """The just-captured step becomes the cache entry of its shape."""
        self._key = (tuple(self._static[0].shape), tuple(self._static[1].shape))
        self._graphs[self._key] = (self.graph, self.segments, self._static)
        self._graphs.move_to_end(self._key)
        self.graph_stats["captures"] += 1

    @property
    def cached_shapes(self) -> int:
        return len(self._graphs)

    def _select(self, src: torch.Tensor, tgt: torch.Tensor) -> None:
        """Make the captured step of this batch shape current: a cache hit,
        or (bucketed) a capture of the new shape, evicting the least recently
        used one when the cache is full. Every rank sees the same global-batch
        shapes in the same order, so every rank captures and evicts alike."""
        key = (tuple(src.shape), tuple(tgt.shape))
        if key == self._key:
            return
        ent = self._graphs.get(key)
        if ent is not None:
            self._graphs.move_to_end(key)
            self.graph, self.segments, self._static = ent
            self._key = key
            return
        if not self.bucketed:
            raise ValueError(f"captured step takes {tuple(self._static[0].shape)} / "
                             f"{tuple(self._static[1].shape)} batches, got {tuple(src.shape)} / "
                             f"{tuple(tgt.shape)}")
        while len(self._graphs) >= max(1, self.graph_cache):
            self._graphs.popitem(last=False)
            self.graph_stats["evictions"] += 1
        self.graph = self.segments = None
        self._static = None
        self._key = None
        if not self.capture(src, tgt, warmup=1):
            raise RuntimeError("bucketed step: capture of a new batch shape failed")

    def choose_dp_mode(self, src: torch.Tensor, tgt: torch.Tensor, steps: int = 8,
                       rounds: int = 3, margin: float = 0.03) -> Dict[str, object]:
        """Data parallel: pick how the step runs on THIS node, by measurement.

        Arms: the segmented graph (collectives issued between graph segments)
        and the eager step; and, where a comm thread exists
        (ddp.COMM_THREAD "auto"), both once more with the collectives issued
        by the host comm thread instead of the process group's own stream
        handoff. Each arm is timed in interleaved rounds
        (median per arm, MAX over ranks, so every rank takes the same
        decision) and, after its timed steps, the replicas must be bitwise
        equal (DataParallel.verify_replicas raises otherwise: an issue path
        that breaks synchronous DP is an error, not a slower option). The
        segmented graph wins when the host is the bottleneck (eight ranks
        sharing a node's CPUs); the eager step when the host keeps ahead. The
        training state is restored afterwards, so this trains nothing.
        Without a measurement (the step is not captured, DP_AUTOSELECT off)
        an available comm thread is used. Returns {"mode": "seg" | "0",
        "comm_thread": bool, "reason": "measured" | "unmeasured",
        "<arm>_ms": .., "select_s": seconds this selection took}."""
        ddp = self.ddp
        t_start = time.perf_counter()
        auto_thread = (ddp is not None and ddp.active and ddp.can_thread
                       and _ddp_mod.COMM_THREAD == "auto")
        if auto_thread:
            ddp.use_thread(False)

        def unmeasured(mode: str) -> Dict[str, object]:
            # no start-up measurement: with a comm thread available ("auto")
            # the thread issues the collectives -- it won the one-rank RCCL A/B
            # on MI355X for the eager and the segmented step alike (5.11 vs
            # 5.34 ms, profiles/r4/ab_dp_comm_thread.txt)
            if auto_thread:
                ddp.use_thread(True)
            th = ddp is not None and ddp._thread is not None
            return {"mode": mode, "comm_thread": th, "reason": "unmeasured",
                    "select_s": round(time.perf_counter() - t_start, 3)}

        if not self.capture(src, tgt):
            return unmeasured(self.capture_mode())
        if not (ddp is not None and ddp.active and self.segments is not None) or not DP_AUTOSELECT:
            return unmeasured("seg" if self.segments is not None else self.capture_mode())
        arms = {"seg": (self.segments, ddp._thread is not None)}
        if auto_thread:
            self.segments = None
            ddp.use_thread(True)
            if self.capture(src, tgt):
                arms["seg_thread"] = (self.segments, True)
            ddp.use_thread(False)
        saved = self.snapshot()
        dev = self.model.device

        def timed(run) -> float:
            for _ in range(2):
                run()
            torch.cuda.synchronize()
            ddp.check_quiescent("choose_dp_mode")
            dist.barrier(group=ddp.group)
            t0 = time.perf_counter()
            for _ in range(steps):
                run()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            ddp.verify_replicas()  # the arm kept synchronous DP exact
            return dt

        def seg_run(name):
            segs, th = arms[name]

            def run():
                self.segments = segs
                self(src, tgt)
            return run, th

        # eager arms: the process group's handoff, and (auto) the comm thread
        eager_arms = {"0": False}
        if auto_thread:
            eager_arms["0_thread"] = True
        names = list(arms) + list(eager_arms)
        runs = {k: [] for k in names}
        for _ in range(rounds):
            for k in names:
                if k in eager_arms:
                    self.segments = None
                    ddp.use_thread(eager_arms[k])
                    runs[k].append(timed(lambda: self.eager(src, tgt)))
                else:
                    run, th = seg_run(k)
                    ddp.use_thread(th)  # (a captured graph keeps its own path)
                    runs[k].append(timed(run))
        # median per arm: one noisy round (box clock, host contention) does
        # not decide the mode for the whole run
        med = {k: sorted(v)[len(v) // 2] for k, v in runs.items()}
        t = torch.tensor([med[k] for k in names], dtype=torch.float64, device=dev)
        ddp.check_quiescent("choose_dp_mode")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ddp.group)
        ms = {k: float(v) for k, v in zip(names, t.tolist())}
        self.restore(saved)
        best_seg = min((k for k in names if k not in eager_arms), key=lambda k: ms[k])
        best_eager = min(eager_arms, key=lambda k: ms[k])
        if ms[best_eager] < ms[best_seg] * (1.0 - margin):
            self.segments = None
            self._static = None
            th = eager_arms[best_eager]
            ddp.use_thread(th)
            mode = "0"
        else:
            self.segments, th = arms[best_seg]
            ddp.use_thread(th)
            mode = "seg"
        arms.clear()  # the other captures' graphs are released
        self._graphs.clear()
        self._key = None
        if self.segments is not None:
            self._register()
        torch.cuda.synchronize()
        out = {"mode": mode, "comm_thread": th, "reason": "measured"}
        out.update({f"{k.replace('0', 'eager', 1) if k.startswith('0') else k}_ms": round(v * 1e3, 3)
                    for k, v in ms.items()})
        out["select_s"] = round(time.perf_counter() - t_start, 3)
        return out

    def __call__(self, src: torch.Tensor, tgt: torch.Tensor) -> torch.Tensor:
        if not self.captured:
            return self.eager(src, tgt)
        if src.shape != self._static[0].shape or tgt.shape != self._static[1].shape:
            self._select(src, tgt)
        self.graph_stats["replays"] += 1
        self._static[0].copy_(src, non_blocking=True)
        self._static[1].copy_(tgt, non_blocking=True)
        if self.segments is not None:
            self.segments.replay()
        else:
            self.graph.replay()
        return self.last
