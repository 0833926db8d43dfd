"""Manual Python garbage collection for the training loop.

The eager data-parallel step is close to launch-bound (each rank enqueues
~240 kernels per 5.6 ms step from Python), so a cyclic-GC pass landing inside
a step shows up directly as step-time jitter on that rank -- and a
synchronous all-reduce makes every rank wait for the slowest one. With the
policy on, everything alive after warm-up (model, optimizer, workspaces) is
moved to the permanent generation (gc.freeze), automatic collection is off,
and a young-generation collection runs every `interval` steps at a point the
caller chooses (outside the timed step), so every rank collects on the same
step.

Measured on one MI355X (scripts/gc_ab.sh, profiles/bench/gc_ab_v1.txt):
neutral on the eager data-parallel step within its +-0.2 ms run-to-run
noise (5.64-5.92 ms off vs 5.78-6.00 ms on), so it is opt-in
(TDG_MANUAL_GC=1) until a multi-rank run shows the max-over-ranks jitter it
targets.

No reference counterpart (TF runs its step as a graph, reference
__main__.py:105-132); this is host-side hygiene for the eager Python path.
"""
from __future__ import annotations

import gc
import os


class ManualGC:
    def __init__(self, interval: int = 200, enabled: bool = True):
        self.interval = max(1, int(interval))
        self.enabled = enabled
        self._n = 0
        self._was_enabled = gc.isenabled()
        if enabled:
            gc.collect()
            gc.freeze()
            gc.disable()

    @classmethod
    def from_env(cls) -> "ManualGC":
        """TDG_MANUAL_GC: "1" on (default off); TDG_GC_INTERVAL steps (200)."""
        return cls(interval=int(os.environ.get("TDG_GC_INTERVAL", "200")),
                   enabled=os.environ.get("TDG_MANUAL_GC", "0") == "1")

    def step(self) -> bool:
        """Call once per step outside the timed region; True if it collected."""
        if not self.enabled:
            return False
        self._n += 1
        if self._n % self.interval == 0:
            gc.collect(1)
            return True
        return False

    def close(self) -> None:
        if self.enabled:
            gc.unfreeze()
            if self._was_enabled:
                gc.enable()
            self.enabled = False
