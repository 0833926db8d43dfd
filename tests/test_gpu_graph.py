"""HIP-graph replay of the whole training step equals the eager step.

One GPU: TrainStep.capture() runs warm-up steps eagerly, restores the state
they changed, then captures one step; replays must leave exactly the weights
that the same number of eager steps leave (dropout counter, Adam step and
fp8 scales all live on the device), and capture() itself trains nothing
(opt.iterations counts the replayed steps only). Data parallel (single-rank
RCCL communicator, --force-dp): the segmented graph (collectives issued
eagerly between graph segments, the default multi-GPU step); the 8-GPU RCCL
replay itself is not testable on one GPU."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

STEPS = 3


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(dev):
    g = torch.Generator().manual_seed(7)
    out = []
    for i in range(STEPS + 1):
        src = torch.randint(4, 500, (16, 48), generator=g)
        tgt = torch.randint(4, 400, (16, 41), generator=g)
        src[:, 30 + i:] = 0
        tgt[:, 25 + 2 * i:] = 0
        out.append((src.to(dev), tgt.to(dev)))
    return out


def _run(dev, graph, ddp_factory=None, fp8=False, select_margin=None):
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    kk.AUTOTUNE = False  # identical GEMM configs in both runs
    cfg = model_config("tiny", d_model=256, heads=4, d_ff=1024, src_vocab=500, tgt_vocab=400, dropout=0.1)
    m = Transformer(cfg).build(dev, seed=3)
    opt = Adam(m.store, cfg.d_model, lr=0.003)
    ddp = ddp_factory(m) if ddp_factory else None
    fp8_state = None
    if fp8:
        from tensorflow_distributed_on_gke_amd.ops.fp8 import Fp8State
        fp8_state = Fp8State(m)
    step = TrainStep(m, opt, ddp, workers=1, seed=11, fp8_state=fp8_state)
    bs = _batches(dev)
    losses = []
    if graph and select_margin is not None:
        # measured choice between the segmented graph and the eager step; the
        # margin forces either outcome. Neither the capture nor the timed
        # steps may train anything.
        sel = step.choose_dp_mode(*bs[0], steps=2, rounds=1, margin=select_margin)
        step.selected = sel
        assert opt.iterations == 0 and int(step.rt.ctr.item()) == 0
    elif graph:
        assert step.capture(*bs[0], warmup=2)  # warm-up steps are rolled back
        assert opt.iterations == 0 and int(step.rt.ctr.item()) == 0
    for i in range(STEPS + 1):
        losses.append(step(*bs[i]).clone())
    torch.cuda.synchronize()
    assert opt.iterations == STEPS + 1
    return m.store.flat.cpu(), torch.stack(losses).cpu(), step


def test_graph_replay_matches_eager_one_gpu():
    f_e, l_e, _ = _run("cuda", graph=False)
    f_g, l_g, st = _run("cuda", graph=True)
    assert st.graph is not None
    assert torch.isfinite(f_g).all()
    assert torch.equal(l_e, l_g), (l_e, l_g)
    assert torch.equal(f_e, f_g)


def test_graph_replay_matches_eager_fp8():
    f_e, l_e, _ = _run("cuda", graph=False, fp8=True)
    f_g, l_g, st = _run("cuda", graph=True, fp8=True)
    assert st.graph is not None
    assert torch.equal(l_e, l_g), (l_e, l_g)
    assert torch.equal(f_e, f_g)


def _dp_worker(rank, port, out, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0", TDG_DP_GRAPH=mode)
    from tensorflow_distributed_on_gke_amd.parallel import dist as tdist
    from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel

    info = tdist.init_distributed("cuda", force=True)

    def mk(m):
        d = DataParallel(m.store, bucket_mb=1.0, force=True)
        d.broadcast_params(0)
        return d

    res = {}
    for graph in (False, True):
        f, l, st = _run(info.device, graph, mk)
        assert st.ddp is not None and st.ddp.active and len(st.ddp.last_buckets) > 1
        if graph:
            assert st.segments is not None and st.graph is None
            # one issue per span + two wait points (backward's spans, the last span)
            assert st.segments.num_calls == len(st.ddp.last_buckets) + 2, st.segments.items
        res["graph" if graph else "eager"] = (f, l)
    # measured mode selection, each outcome forced by the margin
    for name, margin, want in (("sel_eager", -10.0, "0"), ("sel_seg", 0.99, "seg")):
        f, l, st = _run(info.device, True, mk, select_margin=margin)
        assert st.selected["mode"] == want, st.selected
        assert (st.segments is not None) == (want == "seg")
        assert st.selected["seg_ms"] > 0 and st.selected["eager_ms"] > 0
        # RCCL (one rank): the host comm-thread arm is measured (and its
        # replicas verified) too, and the choice is recorded
        assert st.selected["seg_thread_ms"] > 0 and st.selected["eager_thread_ms"] > 0, st.selected
        assert st.selected["reason"] == "measured" and st.selected["select_s"] > 0
        assert st.selected["comm_thread"] == (st.ddp._thread is not None)
        res[name] = (f, l)
    torch.save({"ef": res["eager"][0], "el": res["eager"][1], "gf": res["graph"][0], "gl": res["graph"][1],
                "sef": res["sel_eager"][0], "ssf": res["sel_seg"][0], "sel": res["sel_eager"][1],
                "ssl": res["sel_seg"][1]}, out)
    tdist.shutdown()


@pytest.mark.parametrize("mode", ["seg"])
def test_dp_step_graph_matches_eager(tmp_path, mode):
    out = str(tmp_path / "dp.pt")
    mp.start_processes(_dp_worker, args=(_port(), out, mode), nprocs=1, join=True, start_method="spawn")
    r = torch.load(out, weights_only=True)
    assert torch.equal(r["el"], r["gl"]), (r["el"], r["gl"])
    assert torch.equal(r["ef"], r["gf"])
    # after a measured mode choice (either outcome) training is unchanged
    for k in ("sef", "ssf"):
        assert torch.equal(r["ef"], r[k]), k
    assert torch.equal(r["el"], r["sel"]) and torch.equal(r["el"], r["ssl"])
