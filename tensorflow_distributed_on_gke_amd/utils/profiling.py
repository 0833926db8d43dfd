"""Observability: device-event step timers, a tokens/s meter, a JSONL metrics
sink and a torch.profiler wrapper.

The reference only timed whole epochs with time.time()
(reference: distributed_training_transformer/__main__.py:150,179-180). Here
each step is bracketed by HIP events recorded on the compute stream — no host
synchronisation in the loop; elapsed times are resolved when the host reads
them (log points). rocprofv3 recipes live in scripts/profile_bench.sh and
scripts/pmc_gemm.sh.
"""
from __future__ import annotations

import json
import os
import time
from contextlib import contextmanager
from typing import Dict, List, Optional

import torch


class StepTimer:
    """Ring of (start, end) HIP events; CPU wall clock when no GPU."""

    def __init__(self, device: torch.device, capacity: int = 1024):
        self.cuda = device.type == "cuda"
        self.capacity = capacity
        self._pending: List = []
        self._done: List[float] = []
        self._t0: Optional[float] = None

    def start(self) -> None:
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._pending.append([ev, None])
        else:
            self._t0 = time.perf_counter()

    def stop(self) -> None:
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self._pending[-1][1] = ev
            if len(self._pending) > self.capacity:
                self._resolve(self._pending[: len(self._pending) // 2])
                self._pending = self._pending[len(self._pending) // 2:]
        else:
            self._done.append((time.perf_counter() - self._t0) * 1e3)

    def _resolve(self, pairs) -> None:
        for s, e in pairs:
            if e is not None:
                e.synchronize()
                self._done.append(s.elapsed_time(e))

    def drain(self) -> List[float]:
        """Step times in ms since the last drain (synchronises on the events)."""
        self._resolve(self._pending)
        self._pending = []
        out, self._done = self._done, []
        return out


def summarize(ms: List[float]) -> Dict[str, float]:
    if not ms:
        return {"steps": 0}
    s = sorted(ms)
    return {"steps": len(s), "mean_ms": sum(s) / len(s), "p50_ms": s[len(s) // 2],
            "p90_ms": s[min(len(s) - 1, int(0.9 * len(s)))], "max_ms": s[-1]}


class MetricsWriter:
    """Append-only JSONL metrics file (rank 0)."""

    def __init__(self, path: Optional[str]):
        self.path = path
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def write(self, **rec) -> None:
        if not self.path:
            return
        rec.setdefault("time", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")


def tokens_per_second(tokens_per_step: float, ms_per_step: float) -> float:
    return tokens_per_step / (ms_per_step / 1e3) if ms_per_step > 0 else 0.0


@contextmanager
def torch_profile(out_dir: Optional[str], active: int = 5):
    """`with torch_profile(dir) as p: ... p.step()` — Chrome trace of HIP
    kernels (roctracer); a no-op when out_dir is None."""
    if not out_dir:
        class _Null:
            def step(self):
                pass
        yield _Null()
        return
    from torch.profiler import ProfilerActivity, profile, schedule, tensorboard_trace_handler

    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])
    with profile(activities=acts, schedule=schedule(wait=1, warmup=1, active=active),
                 on_trace_ready=tensorboard_trace_handler(out_dir)) as p:
        yield p
