"""Flat parameter storage.

All trainable parameters live in ONE flat f32 master buffer, with one flat f32
gradient buffer and (on GPU) one flat bf16 compute-copy ("shadow") at the same
offsets. This is what lets:
  * the optimizer be a single multi-tensor Adam kernel over the whole model,
  * data-parallel gradient all-reduce run on contiguous buckets of the grad
    buffer (no per-tensor packing), launched as soon as a bucket's last
    gradient is produced during backward,
  * checkpoints stream straight out of one host copy.

Layout: parameters are placed in REVERSE order of registration (registration
follows the forward pass), so gradients — produced roughly in reverse forward
order — fill the buffer front to back and buckets complete early in backward.
Every parameter starts on a 64-element boundary (256-byte aligned f32,
128-byte aligned bf16: vector loads in every kernel).

Parameters are named by their TensorFlow checkpoint key stem (reference
variable names) plus a layout descriptor so the TensorBundle
writer can emit the reference's exact keys and [in, out] Dense layout.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

import torch

ALIGN = 64


@dataclass
class TFSlot:
    """How one TF checkpoint variable maps onto (a slice of) an internal param.

    internal[rows] (optionally transposed) == tf variable."""

    key: str
    row0: int
    row1: int
    transpose: bool


@dataclass
class Param:
    name: str
    shape: tuple
    init: Callable[[torch.Tensor, torch.Generator], None]
    tf: List[TFSlot] = field(default_factory=list)
    index: int = -1
    offset: int = 0
    numel: int = 0
    master: Optional[torch.Tensor] = None
    grad: Optional[torch.Tensor] = None
    compute: Optional[torch.Tensor] = None  # bf16 shadow (GPU) / master (CPU)
    compute_t: Optional[torch.Tensor] = None  # transposed bf16 copy (ParamStore.add_transposed)
    compute_t_stale: bool = False  # compute_t lags the compute copy (re-transposes paused)

    def __repr__(self) -> str:  # pragma: no cover
        return f"Param({self.name}, {self.shape}, off={self.offset})"


def glorot_uniform(fan_in: int, fan_out: int):
    lim = math.sqrt(6.0 / (fan_in + fan_out))

    def f(t: torch.Tensor, g: torch.Generator):
        t.uniform_(-lim, lim, generator=g)

    return f


def glorot_blocks(block_rows: int, fan_in: int, fan_out: int):
    """Fused [k*out, in] weight made of k independently glorot-initialised
    [out, in] blocks (Keras initialises each Dense separately)."""
    lim = math.sqrt(6.0 / (fan_in + fan_out))

    def f(t: torch.Tensor, g: torch.Generator):
        for r in range(0, t.shape[0], block_rows):
            t[r : r + block_rows].uniform_(-lim, lim, generator=g)

    return f


def uniform(lo: float, hi: float):
    def f(t, g):
        t.uniform_(lo, hi, generator=g)

    return f


def const(v: float):
    def f(t, g):
        t.fill_(v)

    return f


class ParamStore:
    def __init__(self):
        self.params: List[Param] = []
        self.by_name: Dict[str, Param] = {}
        self.flat: Optional[torch.Tensor] = None
        self.flat_grad: Optional[torch.Tensor] = None
        self.flat_compute: Optional[torch.Tensor] = None
        self.total = 0
        self.device = torch.device("cpu")
        self.compute_dtype = torch.float32
        self._ready_hooks: List[Callable[[Param], None]] = []
        self._release_hooks: List[Callable[[], None]] = []
        self._sync_hooks: List[Callable[[], None]] = []
        self.transposed: List[Param] = []  # weights with a transposed compute copy
        # paused: nothing reads the transposed copies (the fp8 FFN backward
        # runs on the e4m3 weights), so the optimizer skips re-transposing
        # them and marks them stale (Param.compute_t_stale) -- a bf16 FFN
        # backward then takes the untransposed (NN) dgrad
        self.transposed_paused = False
        # autograd anchor: gives layers whose only inputs are token ids a
        # tensor that requires grad, so backward reaches them.
        self.anchor = torch.zeros((), requires_grad=True)

    def add(self, name: str, shape: Sequence[int], init, tf: Optional[List[TFSlot]] = None) -> Param:
        if name in self.by_name:
            raise ValueError(f"duplicate parameter {name}")
        p = Param(name=name, shape=tuple(int(s) for s in shape), init=init, tf=tf or [])
        p.index = len(self.params)
        p.numel = int(math.prod(p.shape))
        self.params.append(p)
        self.by_name[name] = p
        return p

    # ------------------------------------------------------------------ build
    def finalize(self, device, compute_dtype=torch.bfloat16, seed: int = 0) -> None:
        device = torch.device(device)
        self.device = device
        self.compute_dtype = compute_dtype if device.type == "cuda" else torch.float32
        off = 0
        for p in reversed(self.params):
            p.offset = off
            off += (p.numel + ALIGN - 1) // ALIGN * ALIGN
        self.total = off
        host = torch.zeros(self.total, dtype=torch.float32)
        g = torch.Generator().manual_seed(seed)
        for p in self.params:  # init in registration (forward) order: stable across layouts
            v = host[p.offset : p.offset + p.numel].view(p.shape)
            p.init(v, g)
        self.flat = host.to(device)
        self.flat_grad = torch.zeros(self.total, dtype=torch.float32, device=device)
        if self.compute_dtype != torch.float32:
            self.flat_compute = torch.empty(self.total, dtype=self.compute_dtype, device=device)
        for p in self.params:
            p.master = self.flat[p.offset : p.offset + p.numel].view(p.shape)
            p.grad = self.flat_grad[p.offset : p.offset + p.numel].view(p.shape)
            if self.flat_compute is not None:
                p.compute = self.flat_compute[p.offset : p.offset + p.numel].view(p.shape)
            else:
                p.compute = p.master
        self.anchor = torch.zeros((), requires_grad=True, device=device)
        self.refresh_compute()

    def refresh_compute(self) -> None:
        """Re-derive the bf16 compute copy from the f32 masters."""
        if self.flat_compute is None:
            return
        from tensorflow_distributed_on_gke_amd.ops import _ext

        _ext.C().to_bf16(self.flat, self.flat_compute)
        self.refresh_transposed()

    # ------------------------------------------------------------------ transposed copies
    def add_transposed(self, p: Param) -> None:
        """Keep a transposed bf16 copy p.compute_t [in, out] of a 2-D weight
        (GPU): kernels that read the weight K-contiguous the other way round
        (the relu-backward dgrad of the FFN output projection) use it. Every
        writer of the compute copy refreshes it (refresh_compute, the optimizer)."""
        if self.flat_compute is None or p.compute_t is not None:
            return
        p.compute_t = torch.empty(p.shape[1], p.shape[0], dtype=self.compute_dtype,
                                  device=self.device)
        self.transposed.append(p)
        self.refresh_transposed()

    def refresh_transposed(self, start: int = 0, end: Optional[int] = None) -> None:
        """Re-transpose the registered weights lying in flat[start:end]."""
        if not self.transposed:
            return
        if self.transposed_paused:
            for p in self.transposed:
                p.compute_t_stale = True
            return
        end = self.total if end is None else end
        todo = [p for p in self.transposed if p.offset >= start and p.offset + p.numel <= end]
        groups: Dict[tuple, List[Param]] = {}
        for p in todo:
            groups.setdefault(tuple(p.shape), []).append(p)
        from tensorflow_distributed_on_gke_amd.ops import kernels as K

        for ps in groups.values():
            K.transpose_grouped([p.compute for p in ps], [p.compute_t for p in ps])
        for p in todo:
            p.compute_t_stale = False

    # ------------------------------------------------------------------ grads
    def on_grad_ready(self, fn: Callable[[Param], None]) -> None:
        self._ready_hooks.append(fn)

    def clear_grad_hooks(self) -> None:
        self._ready_hooks.clear()

    def grad_ready(self, p: Param) -> None:
        for h in self._ready_hooks:
            h(p)

    def on_grad_sync(self, fn: Callable[[], None]) -> None:
        self._sync_hooks.append(fn)

    def grad_sync(self) -> None:
        """A batch of gradients just became final together (one flush of the
        deferred weight-gradient GEMMs): a natural collective boundary."""
        for h in self._sync_hooks:
            h()

    def on_release(self, fn: Callable[[], None]) -> None:
        self._release_hooks.append(fn)

    def release_point(self) -> None:
        """Called by the model during backward at a point after which no
        kernel still to be issued in this backward reads any parameter whose
        gradient is already final: from here on those parameters may be
        updated concurrently with the rest of backward."""
        for h in self._release_hooks:
            h()

    def zero_grad(self) -> None:
        self.flat_grad.zero_()

    def num_params(self) -> int:
        return sum(p.numel for p in self.params)

    # ------------------------------------------------------------------ state
    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {p.name: p.master.detach().cpu().clone() for p in self.params}

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
        missing = [p.name for p in self.params if p.name not in sd]
        if strict and missing:
            raise KeyError(f"missing parameters: {missing[:5]}...")
        for p in self.params:
            if p.name in sd:
                t = sd[p.name]
                if tuple(t.shape) != p.shape:
                    raise ValueError(f"{p.name}: shape {tuple(t.shape)} != {p.shape}")
                p.master.copy_(t.to(p.master.dtype))
        self.refresh_compute()
