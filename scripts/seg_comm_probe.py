#!/usr/bin/env python3
"""Diagnostic: where the segmented data-parallel step's extra time on one rank
goes. The same captured step (8 graphs, 7 collective calls) with
  real     -- the single-rank RCCL all-reduce calls (ProcessGroupNCCL),
  noop     -- the collectives replaced by no-ops (numerically identical for one
              rank): the cost of the graph cuts alone,
  events   -- no collective, only ProcessGroupNCCL's stream pattern: the comm
              stream waits for an event recorded on the compute stream, the
              compute stream later waits for an event of the comm stream,
  issue    -- only the first half (record on compute, comm stream waits),
  waitonly -- only the second half (compute waits on an idle stream's event),
  record   -- only the event record on the compute stream (nobody waits).
Interleaved rounds, ms/step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for k, v in dict(MASTER_ADDR="127.0.0.1", MASTER_PORT="29613", RANK="0", WORLD_SIZE="1",
                 LOCAL_RANK="0").items():
    os.environ.setdefault(k, v)

import torch  # noqa: E402

from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs  # noqa: E402
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config  # noqa: E402
from tensorflow_distributed_on_gke_amd.parallel import dist as tdist  # noqa: E402
from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel, Pending  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.optim import Adam  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.step import TrainStep  # noqa: E402

_SIDE = {}


def _side():
    if "s" not in _SIDE:
        _SIDE["s"] = torch.cuda.Stream()
        _SIDE["idle"] = torch.cuda.Event()
        _SIDE["idle"].record(torch.cuda.Stream())
    return _SIDE["s"]


class _Work:
    def __init__(self, mode):
        self.mode = mode
        self.ev = None
        if mode == "record":
            self.ev = torch.cuda.Event()
            self.ev.record(torch.cuda.current_stream())
        if mode in ("events", "issue"):
            s = _side()
            s.wait_stream(torch.cuda.current_stream())
            self.ev = torch.cuda.Event()
            self.ev.record(s)

    def wait(self):
        if self.mode == "events":
            torch.cuda.current_stream().wait_event(self.ev)
        elif self.mode == "waitonly":
            _side()
            torch.cuda.current_stream().wait_event(_SIDE["idle"])
        return True


def build(mode):
    m = Transformer(model_config("base")).build("cuda", seed=0)
    opt = Adam(m.store, m.cfg.d_model)
    ddp = DataParallel(m.store, bucket_mb=64.0, force=True)
    if mode != "real":
        def issue(t):
            h = Pending(ddp)

            def go():
                h.work = _Work(mode)
            if ddp.recorder is not None:
                ddp.recorder.cut(go)
            else:
                go()
            return h
        ddp.all_reduce_async = issue
    return TrainStep(m, opt, ddp, workers=1, seed=1)


def main():
    tdist.init_distributed(force=True)
    data = SyntheticPairs(64, 128, 129, 7765, 7010, seed=0)
    src, tgt = (t.cuda() for t in data.batch(0))
    modes = ("real", "noop", "events", "issue", "waitonly", "record")
    steps = {}
    for mode in modes:
        st = build(mode)
        assert st.capture(src, tgt)
        steps[mode] = st
    res = {k: [] for k in modes}
    for _ in range(3):
        for mode in modes:
            st = steps[mode]
            for _ in range(5):
                st(src, tgt)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(30):
                st(src, tgt)
            torch.cuda.synchronize()
            res[mode].append((time.perf_counter() - t0) / 30 * 1e3)
    for mode in modes:
        print(f"{mode:9s}", [round(x, 3) for x in res[mode]])
    seg = steps["real"].segments
    print("graphs/calls per step:", seg.num_graphs, seg.num_calls)
    tdist.shutdown()


if __name__ == "__main__":
    main()
