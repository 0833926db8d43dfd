"""Keras-semantics Adam over the flat master buffer.

GPU: one multi-tensor kernel (csrc/kernels/adam.hip) for the whole model,
reading the step counter and evaluating the Noam schedule on device, fused with
the bf16 shadow refresh and gradient zeroing. CPU: the same update in PyTorch.

Reference: distributed_training_transformer/__main__.py:72-73
(Adam(learning_rate=NoamSchedule(d_model), beta_1=0.9, beta_2=0.98, epsilon=1e-9)).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

from tensorflow_distributed_on_gke_amd.models.params import ParamStore
from tensorflow_distributed_on_gke_amd.ops import kernels as K
from tensorflow_distributed_on_gke_amd.train.schedule import noam_lr


# whole-buffer steps through the contiguous-chunk kernel (adam_chunk_kernel:
# one 4096-parameter chunk per workgroup) instead of the grid-strided one
ADAM_CHUNKED = True


class Adam:
    def __init__(self, store: ParamStore, d_model: int, warmup: float = 4000.0, beta1: float = 0.9,
                 beta2: float = 0.98, eps: float = 1e-9, lr: Optional[float] = None,
                 weight_decay: float = 0.0):
        self.store = store
        self.d_model = d_model
        self.warmup = warmup
        self.beta1, self.beta2, self.eps = beta1, beta2, eps
        self.lr_const = lr  # None -> Noam schedule
        self.weight_decay = weight_decay
        dev = store.flat.device
        self.m = torch.zeros_like(store.flat)
        self.v = torch.zeros_like(store.flat)
        # Keras `iterations`: device-resident so the step is graph-capturable
        self.step = torch.zeros(1, dtype=torch.int64, device=dev)
        # zero the consumed gradient (so the next backward may accumulate).
        # TrainStep turns it off on the GPU, where every gradient writer of a
        # non-accumulating backward overwrites (beta = 0): 4 B/param of HBM
        # writes less in the bandwidth-bound optimizer.
        self.zero_grad = True

    @property
    def iterations(self) -> int:
        return int(self.step.item())

    def lr_at(self, step: int) -> float:
        if self.lr_const is not None:
            return self.lr_const
        return noam_lr(step, self.d_model, self.warmup)

    def apply(self, grad_scale: float = 1.0, fp8w=None) -> bool:
        """The whole step. fp8w (ops.fp8.Fp8Weights): also refresh its e4m3
        weight copies from the updated weights in the same pass (GPU; returns
        False -- nothing done -- when its chunk table is unavailable)."""
        s = self.store
        if fp8w is not None:
            chunks = fp8w.adam_chunks(s) if s.flat.is_cuda and s.flat_compute is not None else None
            if chunks is None:
                return False
            K.adam_chunks(s.flat, s.flat_grad, self.m, self.v, s.flat_compute, chunks, self.step,
                          self.beta1, self.beta2, self.eps, self.lr_const or 0.0, float(self.d_model),
                          float(self.warmup), 1.0 * grad_scale, self.weight_decay,
                          0 if self.lr_const is not None else 1, self.zero_grad, True,
                          fp8w.meta.scale, fp8w.meta.amax)
            s.refresh_transposed(0, s.total)
            return True
        self.apply_range(0, self.store.total, grad_scale, inc_step=True)
        return True

    def apply_range(self, start: int, end: int, grad_scale: float = 1.0, inc_step: bool = True) -> None:
        """Update flat[start:end] only (one data-parallel bucket, as soon as its
        all-reduce is done). Every range of a step reads the same step
        counter; exactly one call per step (the last) passes inc_step."""
        s = self.store
        sl = slice(start, end)
        if (s.flat.is_cuda and ADAM_CHUNKED and s.flat_compute is not None and s.total < (1 << 28)
                and start % 4 == 0 and end % 4 == 0 and end > start):
            tabs = self.__dict__.setdefault("_range_chunks", {})
            if (start, end) not in tabs and torch.cuda.is_current_stream_capturing():
                tabs = None  # (tables are built by the eager warm-up steps, not in a capture)
        else:
            tabs = None
        if tabs is not None:
            if (start, end) not in tabs:
                rows = [(c0, min(4096, end - c0), -1, 0) for c0 in range(start, end, 4096)]
                from tensorflow_distributed_on_gke_amd.ops.fp8 import validate_chunk_table
                validate_chunk_table(rows, s.total, 1)
                tabs[(start, end)] = torch.tensor(rows, dtype=torch.int64, device=s.flat.device)
            if getattr(self, "_no8", None) is None:
                self._no8 = (torch.ones(1, device=s.flat.device),
                             torch.zeros(2048, dtype=torch.int32, device=s.flat.device))
            K.adam_chunks(s.flat, s.flat_grad, self.m, self.v, s.flat_compute, tabs[(start, end)],
                          self.step, self.beta1, self.beta2, self.eps, self.lr_const or 0.0,
                          float(self.d_model), float(self.warmup), grad_scale, self.weight_decay,
                          0 if self.lr_const is not None else 1, self.zero_grad, inc_step, *self._no8)
            s.refresh_transposed(start, end)
            return
        if s.flat.is_cuda:
            K.adam(s.flat[sl], s.flat_grad[sl], self.m[sl], self.v[sl],
                   s.flat_compute[sl] if s.flat_compute is not None else None, self.step,
                   self.beta1, self.beta2, self.eps, self.lr_const or 0.0, float(self.d_model),
                   float(self.warmup), grad_scale, self.weight_decay,
                   0 if self.lr_const is not None else 1, self.zero_grad, inc_step)
            s.refresh_transposed(start, end)  # transposed compute copies of updated weights
            return
        step = int(self.step.item())
        lr = self.lr_at(step)
        t = step + 1
        lr_t = lr * math.sqrt(1 - self.beta2 ** t) / (1 - self.beta1 ** t)
        p, g, m, v = s.flat[sl], s.flat_grad[sl], self.m[sl], self.v[sl]
        g = g * grad_scale
        m.add_((g - m) * (1 - self.beta1))
        v.add_((g * g - v) * (1 - self.beta2))
        p.sub_(lr_t * m / (v.sqrt() + self.eps) + lr * self.weight_decay * p)
        s.flat_grad[sl].zero_()
        if inc_step:
            self.step += 1

    def advance_step(self) -> None:
        """Keras `iterations += 1` after a step applied as several ranges."""
        self.step += 1

    def state_dict(self) -> dict:
        return {"m": self.m.detach().cpu(), "v": self.v.detach().cpu(),
                "iterations": torch.tensor(self.iterations)}

    def load_state_dict(self, sd: dict) -> None:
        self.m.copy_(sd["m"])
        self.v.copy_(sd["v"])
        self.step.fill_(int(sd["iterations"]))
