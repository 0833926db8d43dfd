"""Synthetic translation pairs (replaces the TFDS ted_hrlr_translate pipeline,
reference: distributed_training_transformer/english_portugese_dataset.py:21-51).

Batches have the reference's shape conventions: int64 [B, S] source and
[B, T+1] target ([START] ... [END], right-padded with PAD=0; the train step
splits the target into decoder input tgt[:, :-1] and labels tgt[:, 1:]), the
reference vocabulary sizes (pt 7765 / en 7010) and a per-rank disjoint,
deterministic stream (the AutoShardPolicy.DATA analogue). Generation runs in
the native host runtime (`_native.Prefetcher`: C++ worker threads, N batches
ahead) into pinned host buffers, so the host->GPU copy is asynchronous.
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import torch

from tensorflow_distributed_on_gke_amd.ops._ext import native

START_ID, END_ID = 2, 3


class SyntheticPairs:
    def __init__(self, batch: int, src_len: int, tgt_len: int, src_vocab: int = 7765,
                 tgt_vocab: int = 7010, seed: int = 0, rank: int = 0, world: int = 1,
                 min_len: int = 0, copy_task: bool = False, prefetch: int = 4, threads: int = 2,
                 pin: bool = False):
        n = native()
        c = n.SynthConfig()
        c.seed, c.rank, c.world = int(seed), int(rank), int(world)
        c.batch, c.src_len, c.tgt_len = int(batch), int(src_len), int(tgt_len)
        c.src_vocab, c.tgt_vocab = int(src_vocab), int(tgt_vocab)
        c.min_len, c.copy_task = int(min_len), int(bool(copy_task))
        c.start_id, c.end_id = START_ID, END_ID
        self.cfg = c
        self.pin = pin and torch.cuda.is_available()
        self._prefetch = prefetch
        self._threads = threads
        self._pf = None
        self._next = 0

    @property
    def shapes(self) -> Tuple[Tuple[int, int], Tuple[int, int]]:
        return (self.cfg.batch, self.cfg.src_len), (self.cfg.batch, self.cfg.tgt_len)

    def _alloc(self):
        (b, s), (_, t) = self.shapes
        src = torch.empty(b, s, dtype=torch.int64, pin_memory=self.pin)
        tgt = torch.empty(b, t, dtype=torch.int64, pin_memory=self.pin)
        return src, tgt

    def batch(self, step: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """Random access: batch number `step` of this rank's stream."""
        src, tgt = self._alloc()
        native().synth_fill(self.cfg, int(step), src.data_ptr(), tgt.data_ptr())
        return src, tgt

    def next(self, out: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
        """Sequential access through the background prefetcher."""
        if self._pf is None:
            self._pf = native().Prefetcher(self.cfg, self._prefetch, self._threads)
        src, tgt = out if out is not None else self._alloc()
        self._pf.get(self._next, src.data_ptr(), tgt.data_ptr())
        self._next += 1
        return src, tgt

    def seek(self, step: int) -> None:
        self._next = int(step)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        while True:
            yield self.next()
