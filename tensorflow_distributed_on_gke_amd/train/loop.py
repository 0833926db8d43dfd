"""Epoch training loop: logging, validation, snapshots, warm start, resume,
fault injection.

Reference: distributed_training_transformer/__main__.py:34-186. Behaviour kept:
  * per-replica loss = token-mean CE / workers, summed over replicas
    (`strategy.reduce(SUM)`), train loss printed as the running sum / batches,
    accuracy a running mean of per-replica ratios (__main__.py:75-132);
  * "Epoch {e} Batch {b} Loss {:.4f} Accuracy {:.4f}" every 50 batches,
    an epoch summary and "Time taken for 1 epoch: {:.2f} secs"
    (__main__.py:149-180);
  * validation with workers_count=1 (__main__.py:134-137);
  * the chief takes an initial snapshot and one every 5 epochs through the
    ModelUploader (__main__.py:139-169);
  * optional warm start from a weights prefix (__main__.py:87, which always
    loaded saved_weights/2/model_weights);
  * optional idle mode after training (__main__.py:183-186).
Extensions: resume from the newest local training state (weights + Adam
slots + epoch) written by the chief every epoch, broadcast to all ranks; HIP
graph capture of the step; tokens/s in the epoch line; `kill_at_step`
failure injection for the launcher's failure-detection tests.

Metric reads are the only host syncs: the device accumulators are summed over
ranks (one small all-reduce) at log points, not every step.
"""
from __future__ import annotations

import os
import sys
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import torch
import torch.distributed as dist

from tensorflow_distributed_on_gke_amd.checkpoint import bundle
from tensorflow_distributed_on_gke_amd.checkpoint.uploader import ModelUploader, make_storage
from tensorflow_distributed_on_gke_amd.config import Settings
from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
from tensorflow_distributed_on_gke_amd.models.layers import RunCtx
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
from tensorflow_distributed_on_gke_amd.ops import kernels as K
from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel
from tensorflow_distributed_on_gke_amd.parallel.dist import DistInfo
from tensorflow_distributed_on_gke_amd.train.optim import Adam
from tensorflow_distributed_on_gke_amd.train.step import TrainStep
from tensorflow_distributed_on_gke_amd.utils.profiling import MetricsWriter, StepTimer, summarize, torch_profile

RESUME_DIR = "resume"
RESUME_PREFIX = "model_weights"


def build_model(s: Settings, device) -> Transformer:
    over = {k: getattr(s, k) for k in ("layers", "d_model", "heads", "d_ff") if getattr(s, k) is not None}
    cfg = model_config(s.preset, src_vocab=s.src_vocab, tgt_vocab=s.tgt_vocab, dropout=s.dropout,
                       label_smoothing=s.label_smoothing,
                       max_src_len=max(s.max_len, s.src_len), max_tgt_len=max(s.max_len, s.tgt_len + 1),
                       **over)
    return Transformer(cfg).build(device, seed=s.seed)


@dataclass
class EpochStats:
    epoch: int
    train_loss: float
    train_acc: float
    test_loss: float
    test_acc: float
    seconds: float
    tokens_per_s: float


@dataclass
class Trainer:
    settings: Settings
    info: DistInfo
    log: Callable[[str], None] = print
    history: List[EpochStats] = field(default_factory=list)

    def __post_init__(self):
        s, info = self.settings, self.info
        if s.worker_count != info.world and info.chief:
            # the reference used worker_count both as expected size and loss
            # divisor; the runtime world size wins
            self.log(f"note: settings.worker_count={s.worker_count} but world size is {info.world}; "
                     f"using {info.world}")
        self.tokenizers = None
        if s.data == "text":
            # vocabulary sizes come from the tokenizers (reference __main__.py:32-35)
            from tensorflow_distributed_on_gke_amd.data.text import build_tokenizers
            if not s.train_file:
                raise ValueError("data=text needs train_file")
            self.tokenizers = build_tokenizers(s.train_file, s.src_vocab, s.tgt_vocab,
                                               cache_dir=s.temporary_directory if info.chief else None,
                                               src_path=s.src_tokenizer, tgt_path=s.tgt_tokenizer)
            s.src_vocab, s.tgt_vocab = self.tokenizers[0].vocab_size, self.tokenizers[1].vocab_size
        elif s.data != "synthetic":
            raise ValueError(f"unknown data source {s.data!r} (synthetic | text)")
        self.model = build_model(s, info.device)
        self.opt = Adam(self.model.store, self.model.cfg.d_model, warmup=s.warmup_steps, beta1=s.beta1,
                        beta2=s.beta2, eps=s.epsilon, lr=s.learning_rate)
        comm = torch.bfloat16 if s.grad_comm_dtype == "bf16" else None
        self.ddp = (DataParallel(self.model.store, bucket_mb=s.bucket_mb, comm_dtype=comm)
                    if info.world > 1 else None)
        self.fp8 = None
        if s.dtype == "fp8" and info.device.type == "cuda":
            from tensorflow_distributed_on_gke_amd.ops.fp8 import Fp8State
            self.fp8 = Fp8State(self.model)
        self.step_fn = TrainStep(self.model, self.opt, self.ddp, workers=info.world, seed=s.seed + 17,
                                 fp8_state=self.fp8, loss_mode=s.loss_mode)
        # summed accuracy over replicas: a mean of per-replica ratios, or (global
        # token mean) already the global ratio
        self._acc_div = 1 if self.step_fn.global_mean else info.world
        if self.tokenizers is not None:
            from tensorflow_distributed_on_gke_amd.data.text import TextPairs
            st, tt = self.tokenizers
            # (hip_graph: batches padded to length buckets, one captured step each)
            bucket = s.graph_bucket if s.hip_graph and info.device.type == "cuda" else 1
            self.train_data = TextPairs(s.train_file, st, tt, s.local_batch_size, info.rank, info.world,
                                        seed=s.seed, shuffle_buffer=s.shuffle_buffer, max_len=s.max_len,
                                        pin=info.device.type == "cuda", bucket=bucket)
            self.val_data = TextPairs(s.validation_file or s.train_file, st, tt, s.local_batch_size,
                                      info.rank, info.world, seed=s.seed, shuffle=False,
                                      max_len=s.max_len)
            s.steps_per_epoch = self.train_data.steps_per_epoch  # one pass per epoch
            s.validation_steps = self.val_data.steps_per_epoch
        else:
            self.train_data = SyntheticPairs(s.local_batch_size, s.src_len, s.tgt_len + 1, s.src_vocab,
                                             s.tgt_vocab, seed=s.seed, rank=info.rank, world=info.world,
                                             min_len=s.min_len, copy_task=s.copy_task,
                                             pin=info.device.type == "cuda")
            self.val_data = SyntheticPairs(s.local_batch_size, s.src_len, s.tgt_len + 1, s.src_vocab,
                                           s.tgt_vocab, seed=s.seed + 1_000_003, rank=info.rank,
                                           world=info.world, min_len=s.min_len, copy_task=s.copy_task)
        self.start_epoch = 0
        self.uploader: Optional[ModelUploader] = None
        self.global_step = 0
        self.timer = StepTimer(info.device)
        self.metrics = MetricsWriter(s.metrics_file if info.chief else None)

    # ------------------------------------------------------------------ state
    @property
    def resume_prefix(self) -> str:
        return os.path.join(self.settings.temporary_directory, RESUME_DIR, RESUME_PREFIX)

    def _quiet(self, what: str) -> None:
        """No data-parallel collective may be in flight when the main thread
        issues one (parallel/ddp.py check_quiescent)."""
        if self.ddp is not None:
            self.ddp.check_quiescent(what)

    def _broadcast_state(self) -> None:
        if self.info.world > 1:
            self._quiet("broadcast")
            for t in (self.model.store.flat, self.opt.m, self.opt.v, self.opt.step):
                dist.broadcast(t, 0)
            self.model.store.refresh_compute()

    def restore(self) -> None:
        """Warm start / resume on the chief, then broadcast to every rank
        (pods do not share a filesystem)."""
        s = self.settings
        flag = torch.zeros(2, dtype=torch.int64, device=self.info.device)
        if self.info.chief:
            if s.resume and os.path.exists(self.resume_prefix + "_optimizer.index"):
                bundle.load_weights(self.model.store, self.resume_prefix)
                extra = bundle.load_training_state(self.model.store, self.opt, self.resume_prefix)
                flag[0], flag[1] = 1, extra.get("epoch", 0)
                self.log(f"Resuming from {self.resume_prefix} at epoch {extra.get('epoch', 0) + 1}, "
                         f"iteration {self.opt.iterations}")
            elif s.warm_start:
                bundle.load_weights(self.model.store, s.warm_start)
                self.log(f"Warm start from {s.warm_start}")
        if self.info.world > 1:
            dist.broadcast(flag, 0)
        self.start_epoch = int(flag[1].item()) if int(flag[0].item()) else 0
        self._broadcast_state()
        if self.fp8 is not None:
            self.fp8.weights.calibrate()  # weights may have changed (resume / warm start)

    def save_resume_state(self, epochs_done: int) -> None:
        bundle.save_weights(self.model.store, self.resume_prefix)
        bundle.save_training_state(self.model.store, self.opt, self.resume_prefix,
                                   {"epoch": epochs_done, "global_step": self.global_step})

    def _snapshot(self) -> None:
        if self.uploader is None:
            s = self.settings
            storage = make_storage(s.cloud_storage_bucket_name, s.google_cloud_access_key_path,
                                   s.storage_backend, s.storage_root)
            self.uploader = ModelUploader(storage, s.cloud_storage_upload_folder, s.temporary_directory)
        self.uploader.take_snapshot(self.model)

    # ------------------------------------------------------------------ metrics
    def _reduce(self, t: torch.Tensor) -> torch.Tensor:
        t = t.clone()
        if self.info.world > 1:
            self._quiet("metrics all-reduce")
            dist.all_reduce(t)
        return t.cpu()

    def _to_dev(self, batch):
        dev = self.info.device
        return batch[0].to(dev, non_blocking=True), batch[1].to(dev, non_blocking=True)

    def validate(self) -> Dict[str, float]:
        s = self.settings
        rt = RunCtx(training=False, store=None)
        acc = torch.zeros(4, dtype=torch.float32, device=self.info.device)
        out = torch.zeros(2, dtype=torch.float32, device=self.info.device)
        for i in range(s.validation_steps):
            src, tgt = self._to_dev(self.val_data.batch(i))
            # workers_count=1: the test loss is a plain per-replica mean
            self.model.loss_and_backward(src, tgt, rt, 1.0, accum=acc, backward=False, step_out=out)
        a = self._reduce(acc)
        if self.info.device.type == "cuda":
            K.check_trailing_padding()
        n = max(float(a[2]), 1.0)
        return {"loss": float(a[0]) / n, "acc": float(a[1]) / n}

    def _arm_backward_fault(self) -> None:
        """kill_point=backward: this rank exits inside the backward of step
        kill_at_step, after half of the parameters' gradients are final (the
        failure-detection test of a peer dying mid-collective)."""
        s, info = self.settings, self.info
        if s.kill_point not in ("step", "backward"):
            raise ValueError(f"kill_point must be step or backward, got {s.kill_point!r}")
        # the grad-ready hook below runs on the host during an EAGER backward
        # only: a captured step (single HIP graph or the segmented data-parallel
        # graph) replays without it, so with a backward fault armed every rank
        # steps eagerly (fit() skips the capture) -- the fault would otherwise
        # silently never fire
        self._backward_fault_armed = s.kill_at_step >= 0 and s.kill_point == "backward"
        if self._backward_fault_armed and info.chief:
            self.log("fault injection at a backward point: HIP-graph capture disabled for this run")
        if s.kill_at_step < 0 or s.kill_point != "backward" or info.rank != (s.kill_rank % info.world):
            return
        seen = [0]
        half = len(self.model.store.params) // 2

        def hook(_p):
            if self.global_step + 1 != s.kill_at_step:
                return
            seen[0] += 1
            if seen[0] == half:
                self.log(f"fault injection: rank {info.rank} exiting in the backward of step "
                         f"{s.kill_at_step}")
                sys.stdout.flush()
                os._exit(17)

        self.model.store.on_grad_ready(hook)

    # ------------------------------------------------------------------ loop
    def fit(self) -> List[EpochStats]:
        s, info = self.settings, self.info
        self.restore()
        if info.chief and s.snapshot_every_epochs > 0:
            self._snapshot()
            self.log("Initial model snapshot uploaded to " + self.uploader.last_upload_location())
        steps = s.steps_per_epoch
        self.global_step = self.start_epoch * steps
        self.train_data.seek(self.global_step)
        captured = False
        # optional Chrome trace of the first profile_steps + 2 steps (rank 0)
        prof_cm = torch_profile(s.profile_dir if info.chief else None, active=s.profile_steps)
        prof = prof_cm.__enter__()
        prof_left = s.profile_steps + 2 if s.profile_dir and info.chief else 0
        self._arm_backward_fault()
        for epoch in range(self.start_epoch, s.epochs):
            t0 = time.time()
            self.step_fn.accum.zero_()
            epoch_tokens = 0
            for batch in range(steps):
                src, tgt = self._to_dev(self.train_data.next())
                epoch_tokens += (src.shape[1] + tgt.shape[1] - 1) * src.shape[0] * info.world
                if s.hip_graph and info.device.type == "cuda" and not captured \
                        and not self._backward_fault_armed:
                    # capture() restores the state its warm-up steps changed,
                    # so this batch is still trained exactly once (below).
                    # Text data: every new (bucketed) batch shape is captured
                    # the same way when it first arrives (TrainStep._select)
                    self.step_fn.bucketed = s.data == "text"
                    self.step_fn.graph_cache = s.graph_cache
                    if self.ddp is not None and self.ddp.active:
                        sel = self.step_fn.choose_dp_mode(src, tgt)
                        if info.chief:
                            self.log(f"data-parallel step mode: {sel}")
                    elif not self.step_fn.capture(src, tgt) and info.chief:
                        self.log("note: the step runs eagerly")
                    captured = True
                self.timer.start()
                self.step_fn(src, tgt)
                self.timer.stop()
                self.global_step += 1
                if prof_left:
                    prof.step()
                    prof_left -= 1
                    if not prof_left:
                        prof_cm.__exit__(None, None, None)
                if self.ddp is not None and s.check_replicas_every > 0 and \
                        self.global_step % s.check_replicas_every == 0:
                    self.ddp.verify_replicas()
                if s.kill_at_step >= 0 and self.global_step == s.kill_at_step and s.kill_point == "step" and \
                        info.rank == (s.kill_rank % info.world):
                    self.log(f"fault injection: rank {info.rank} exiting at step {self.global_step}")
                    sys.stdout.flush()
                    os._exit(17)
                if batch % s.log_every == 0:
                    if info.device.type == "cuda":
                        K.check_trailing_padding()  # rows with interior PADs (device counter)
                    a = self._reduce(self.step_fn.accum)
                    n = max(float(a[2]) / info.world, 1.0)
                    st = summarize(self.timer.drain())
                    if info.chief:
                        self.log(f"Epoch {epoch + 1} Batch {batch} Loss {float(a[0]) / n:.4f} "
                                 f"Accuracy {float(a[1]) / (n * self._acc_div):.4f}")
                        if self.step_fn.bucketed and self.step_fn.captured:
                            gs = self.step_fn.graph_stats
                            self.log(f"graph cache: {self.step_fn.cached_shapes} batch shapes captured "
                                     f"(captures {gs['captures']}, evictions {gs['evictions']}, "
                                     f"replays {gs['replays']})")
                        self.metrics.write(kind="train", epoch=epoch + 1, batch=batch, step=self.global_step,
                                           loss=float(a[0]) / n, accuracy=float(a[1]) / (n * self._acc_div),
                                           **st)
            a = self._reduce(self.step_fn.accum)
            n = max(float(a[2]) / info.world, 1.0)
            train_loss = float(a[0]) / n
            train_acc = float(a[1]) / (n * self._acc_div)
            if info.device.type == "cuda":
                torch.cuda.synchronize()
            train_time = time.time() - t0
            if info.chief and s.snapshot_every_epochs > 0 and (epoch + 1) % s.snapshot_every_epochs == 0:
                self._snapshot()
                self.log(f"Saving checkpoint for epoch {epoch + 1} at {self.uploader.last_upload_location()}")
            val = self.validate()
            if info.chief and s.resume:
                self.save_resume_state(epoch + 1)
            dt = time.time() - t0
            st = EpochStats(epoch + 1, train_loss, train_acc, val["loss"], val["acc"], dt,
                            epoch_tokens / max(train_time, 1e-9))
            self.history.append(st)
            self.timer.drain()
            self.metrics.write(kind="epoch", **st.__dict__)
            if info.chief:
                self.log(f"Epoch {epoch + 1} Loss {train_loss:.4f} Accuracy {train_acc:.4f} "
                         f"Test Loss {val['loss']:.4f} Test Accuracy {val['acc']:.4f}")
                self.log(f"Time taken for 1 epoch: {dt:.2f} secs ({st.tokens_per_s:,.0f} tokens/s)\n")
            if info.world > 1:
                self._quiet("epoch barrier")
                dist.barrier()
        if prof_left:  # fewer steps than the profile window
            prof_cm.__exit__(None, None, None)
        return self.history


def idle_forever(log=print) -> None:  # pragma: no cover
    log("Training complete, script in idle mode.")
    while True:
        time.sleep(3600)
