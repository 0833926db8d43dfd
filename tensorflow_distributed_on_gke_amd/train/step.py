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
from typing import Optional, Tuple

import torch
import torch.distributed as dist

from tensorflow_distributed_on_gke_amd.models.layers import RunCtx, WgradQueue
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer
from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel
from tensorflow_distributed_on_gke_amd.ops import kernels as K
from tensorflow_distributed_on_gke_amd.ops.streams import join
from tensorflow_distributed_on_gke_amd.train.optim import Adam


# data parallel: weight gradients flushed in wave-sized chunks at layer ends
CHUNKED_WGRAD = os.environ.get("TDG_DP_CHUNKED_WGRAD", "1") != "0"
# tiles per wave of the chunked schedule (one whole-K 256x256 tile per CU);
# overridable so tests can force problems to be cut across launches
WAVE_TILES = int(os.environ.get("TDG_DP_WAVE_TILES", "0"))
# skip the optimizer's gradient zeroing (all GPU gradient writers overwrite)
ZERO_GRAD_FREE = os.environ.get("TDG_ZERO_GRAD_FREE", "1") != "0"


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
            grp = ddp.group
            self._ntok_sum = lambda t: dist.all_reduce(t, group=grp, async_op=True)
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
        self.fp8 = fp8_state
        if dev.type == "cuda" and not self.rt.accumulate and ZERO_GRAD_FREE:
            opt.zero_grad = False  # every GPU gradient writer overwrites
        # data parallel: each bucket's Adam runs as soon as its all-reduce is
        # done. Default "tail": at the end of the step, so the last bucket's
        # all-reduce overlaps the Adam of the others. "1": also mid-backward
        # (decoder side during the encoder's backward) -- on one MI355X with
        # --force-dp that concurrent Adam contended with the encoder backward
        # for more than it hid (6.45 vs 6.34 ms). "0": one Adam after finish.
        mode = os.environ.get("TDG_DP_OVERLAP_OPT", "tail")
        if ddp is not None and ddp.active and fp8_state is None and mode != "0":
            ddp.attach_optimizer(opt, release=mode != "tail")
        # metric accumulators [sum loss, sum acc, n steps, n tokens] (device)
        self.accum = torch.zeros(4, dtype=torch.float32, device=dev)
        self.last = torch.zeros(2, dtype=torch.float32, device=dev)
        self.graph = None
        self._static: Optional[Tuple[torch.Tensor, torch.Tensor]] = None

    def eager(self, src: torch.Tensor, tgt: torch.Tensor) -> torch.Tensor:
        self.model.loss_and_backward(src, tgt, self.rt, self.workers, accum=self.accum,
                                     step_out=self.last, bump_ctr=True, ntok_sum=self._ntok_sum)
        if self.ddp is not None:
            self.ddp.finish()
        else:
            join(self.model.device)  # weight gradients from the side stream
        if self.ddp is None or self.ddp.opt is None:
            self.opt.apply()
        if self.fp8 is not None:
            self.fp8.after_step()  # new scales, then fp8 weight copies
        return self.last

    # ------------------------------------------------------------------ HIP graph
    def capture(self, src: torch.Tensor, tgt: torch.Tensor, warmup: int = 2) -> None:
        """Capture the whole step (fwd+bwd+optimizer) into one HIP graph on
        static input buffers. Warm-up iterations run on a side stream first so
        lazily-allocated workspaces exist before capture."""
        self._static = (src.clone(), tgt.clone())
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.eager(*self._static)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        if self.ddp is not None and self.ddp.active:
            # collectives inside the graph (experimental, TDG_DP_GRAPH=1): no
            # collective of the warm-up may still be pending in the process
            # group's watchdog, and the watchdog's event queries from its own
            # thread must not invalidate this thread's capture
            torch.cuda.synchronize()
            dist.barrier(group=self.ddp.group)
            torch.cuda.synchronize()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                self.eager(*self._static)
        else:
            with torch.cuda.graph(g):
                self.eager(*self._static)
        self.graph = g

    def __call__(self, src: torch.Tensor, tgt: torch.Tensor) -> torch.Tensor:
        if self.graph is None:
            return self.eager(src, tgt)
        self._static[0].copy_(src, non_blocking=True)
        self._static[1].copy_(tgt, non_blocking=True)
        self.graph.replay()
        return self.last
