"""Multi-process data parallelism on CPU (gloo, world_size 2 and 4).

The bucketed, backward-overlapped all-reduce must give exactly the update a
single process computes from both ranks' batches with the reference's loss
scaling (per-replica token mean / workers, gradients SUM-reduced;
reference: distributed_training_transformer/__main__.py:75-132)."""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs
from tensorflow_distributed_on_gke_amd.models.layers import RunCtx
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel, plan_buckets
from tensorflow_distributed_on_gke_amd.train.optim import Adam

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CFG = dict(src_vocab=60, tgt_vocab=50, dropout=0.0)
STEPS = 3
# eps=1 keeps Adam's update ~linear in the gradient: with Keras' eps=1e-9 an
# identically-zero gradient (e.g. the key bias, softmax-invariant) carrying
# 1e-10 summation-order noise is normalised to a full +-lr step
ADAM = dict(lr=0.05, eps=1.0)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(rank, world):
    return SyntheticPairs(4, 10, 11, 60, 50, seed=3, rank=rank, world=world, min_len=3)


def _worker(rank, world, port, out, bucket_mb, comm=None, overlap_opt=0, loss_mode="replica_mean",
            comm_thread=None, jitter_ms=0.0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from tensorflow_distributed_on_gke_amd.train import step as step_mod
    step_mod.DP_OVERLAP_OPT = str(overlap_opt)
    if comm_thread is not None:  # the host comm-thread issue path (ddp.CommThread)
        from tensorflow_distributed_on_gke_amd.parallel import ddp as ddp_mod
        ddp_mod.COMM_THREAD = comm_thread
        ddp_mod.ISSUE_JITTER_MS = jitter_ms
    torch.set_num_threads(1 if world > 4 else 2)
    from tensorflow_distributed_on_gke_amd.parallel import dist as tdist
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    info = tdist.init_distributed("cpu")
    m = Transformer(model_config("tiny", **CFG)).build("cpu", seed=1 + rank)  # ranks differ until broadcast
    opt = Adam(m.store, m.cfg.d_model, **ADAM)
    ddp = DataParallel(m.store, bucket_mb=bucket_mb, comm_dtype=comm)
    ddp.broadcast_params(0)
    early = []  # buckets the optimizer updated at the release point (mid-backward)
    release = ddp._on_release

    def spy():
        before = sum(b.updated for b in ddp.buckets)
        release()
        early.append(sum(b.updated for b in ddp.buckets) - before)

    ddp._on_release = spy
    if comm_thread == "force":
        assert ddp._thread is not None and ddp.comm_choice == "thread"
    step = TrainStep(m, opt, ddp, workers=world, seed=5, loss_mode=loss_mode)
    data = _data(rank, world)
    losses = []
    for i in range(STEPS):
        losses.append(step(*data.batch(i)).clone())
        ddp.verify_replicas()
    saved = m.store.flat[0].clone()
    if rank == 1:  # a diverged replica is detected
        m.store.flat[0] += 1.0
    try:
        ddp.verify_replicas()
        diverged = False
    except RuntimeError:
        diverged = True
    m.store.flat[0] = saved
    torch.save({"flat": m.store.flat.clone(), "loss": torch.stack(losses), "nb": len(ddp.last_buckets),
                "diverged": diverged, "early": torch.tensor(early)},
               f"{out}.{rank}")
    ddp.close()
    tdist.barrier()
    tdist.shutdown()


def _fill(n):
    """ntok_sum stand-in: the global label count, known up front (no handle)."""
    def f(t):
        t.fill_(n)
    return f


def _single_process_reference(world, global_mean=False):
    m = Transformer(model_config("tiny", **CFG)).build("cpu", seed=1)
    opt = Adam(m.store, m.cfg.d_model, **ADAM)
    datas = [_data(r, world) for r in range(world)]
    losses = []
    for i in range(STEPS):
        n_all = float(sum(int((datas[r].batch(i)[1][:, 1:] != 0).sum()) for r in range(world)))
        for r in range(world):
            rt = RunCtx(training=True, dropout=0.0, seed=5, ctr=torch.zeros(1, dtype=torch.int64),
                        accumulate=r > 0)
            if global_mean:  # every part normalised by the whole global batch's label count
                out = m.loss_and_backward(*datas[r].batch(i), rt, 1.0, ntok_sum=_fill(n_all))
            else:
                out = m.loss_and_backward(*datas[r].batch(i), rt, float(world))
            if r == 0:
                losses.append(out.clone())
        opt.apply()
    return m.store.flat, torch.stack(losses)


@pytest.mark.parametrize("bucket_mb,overlap_opt", [(0.05, 1), (64.0, 0)])
def test_dp2_matches_single_process(tmp_path, bucket_mb, overlap_opt):
    world = 2
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _free_port(), out, bucket_mb, None, overlap_opt),
                       nprocs=world, join=True, start_method="spawn")
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    if bucket_mb < 1:
        assert r0["nb"] > 3  # several buckets, launched from inside backward
    if overlap_opt:
        # decoder-side buckets were updated during the encoder's backward
        assert len(r0["early"]) == STEPS and bool((r0["early"] > 0).all()), r0["early"]
    assert torch.equal(r0["flat"], r1["flat"])  # replicas stay identical
    assert r0["diverged"] and r1["diverged"]
    ref_flat, ref_loss = _single_process_reference(world)
    assert not torch.equal(r0["flat"], Transformer(model_config("tiny", **CFG)).build("cpu", seed=1).store.flat)
    assert torch.allclose(r0["flat"], ref_flat, atol=1e-6, rtol=1e-5)
    assert torch.allclose(r0["loss"], ref_loss, atol=1e-6)


def test_dp4_matches_single_process(tmp_path):
    """Four ranks (the rehearsal closest to a node's 8 we can run on CPU):
    small spans launched from inside backward, per-span Adam mid-backward;
    every replica bitwise equal and equal to the single-process update on all
    four ranks' batches."""
    world = 4
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _free_port(), out, 0.05, None, 1),
                       nprocs=world, join=True, start_method="spawn")
    rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    assert rs[0]["nb"] > 3
    for r in rs[1:]:
        assert torch.equal(rs[0]["flat"], r["flat"])
    assert all(r["diverged"] for r in rs)
    ref_flat, ref_loss = _single_process_reference(world)
    assert torch.allclose(rs[0]["flat"], ref_flat, atol=1e-6, rtol=1e-5)
    assert torch.allclose(rs[0]["loss"], ref_loss, atol=1e-6)


@pytest.mark.parametrize("overlap_opt", [1, 0])
def test_dp8_comm_thread_with_issue_jitter(tmp_path, overlap_opt):
    """Eight ranks -- a whole MI355X node's worth -- on the host comm-thread
    issue path (forced over gloo), every collective issued after a random
    per-rank 0-20 ms delay, small spans launched from inside backward (and,
    with overlap_opt, per-span Adam mid-backward): no hang within the
    process-group timeout, every replica bitwise equal after every step
    (verify_replicas in the worker), and the update equal to one process
    running all eight ranks' batches."""
    world = 8
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _free_port(), out, 0.05, None, overlap_opt, "replica_mean",
                                      "force", 20.0),
                       nprocs=world, join=True, start_method="spawn")
    rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    assert rs[0]["nb"] > 3
    for r in rs[1:]:
        assert torch.equal(rs[0]["flat"], r["flat"])
    assert all(r["diverged"] for r in rs)
    ref_flat, ref_loss = _single_process_reference(world)
    assert torch.allclose(rs[0]["flat"], ref_flat, atol=1e-6, rtol=1e-5)
    assert torch.allclose(rs[0]["loss"], ref_loss, atol=1e-6)


def test_dp2_global_token_mean_loss(tmp_path):
    """loss_mode=global_mean: replicas with different label counts give the
    update of one process on the global batch with a plain token-mean loss."""
    world = 2
    d0, d1 = _data(0, world), _data(1, world)
    assert any(int((d0.batch(i)[1][:, 1:] != 0).sum()) != int((d1.batch(i)[1][:, 1:] != 0).sum())
               for i in range(STEPS))
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _free_port(), out, 64.0, None, 0, "global_mean"),
                       nprocs=world, join=True, start_method="spawn")
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    assert torch.equal(r0["flat"], r1["flat"])
    ref_flat, ref_loss = _single_process_reference(world, global_mean=True)
    rep_flat, _ = _single_process_reference(world)
    assert torch.allclose(r0["flat"], ref_flat, atol=1e-6, rtol=1e-5)
    assert not torch.allclose(ref_flat, rep_flat, atol=1e-6, rtol=1e-5)  # the modes differ
    assert torch.allclose(r0["loss"], ref_loss, atol=1e-6)


def test_dp2_bf16_gradient_comm(tmp_path):
    world = 2
    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _free_port(), out, 0.05, torch.bfloat16), nprocs=world,
                       join=True, start_method="spawn")
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    assert torch.equal(r0["flat"], r1["flat"])
    ref_flat, _ = _single_process_reference(world)
    init = Transformer(model_config("tiny", **CFG)).build("cpu", seed=1).store.flat
    # bf16 gradients: the update matches the f32 one to bf16 precision
    rel = (r0["flat"] - ref_flat).norm() / (ref_flat - init).norm()
    assert rel < 2e-2, rel


def test_plan_buckets_cover_flat_buffer():
    m = Transformer(model_config("tiny", **CFG)).build("cpu", seed=0)
    for mb in (0.01, 0.1, 1.0, 100.0):
        bs = plan_buckets(m.store, int(mb * 2 ** 20))
        assert bs[0].start == 0 and bs[-1].end == m.store.total
        for a, b in zip(bs, bs[1:]):
            assert a.end == b.start
        idx = sorted(i for b in bs for i in b.params)
        assert idx == list(range(len(m.store.params)))
        for b in bs[:-1]:
            assert (b.end - b.start) * 4 >= mb * 2 ** 20


def _frontier_dp(m, bucket_mb, min_mb):
    """A DataParallel whose collectives are recorded instead of launched."""
    dp = DataParallel(m.store, bucket_mb=bucket_mb, min_mb=min_mb)
    dp.active = True
    launched = []

    class _Done:
        def wait(self):
            pass

    def fake_launch(b):
        launched.append((b.start, b.end))
        b.work = (_Done(), None, None)

    dp._launch = fake_launch
    m.store.clear_grad_hooks()
    m.store.on_grad_ready(dp._on_ready)
    m.store.on_grad_sync(dp._on_sync)
    return dp, launched


def test_frontier_spans_follow_completion_order():
    """Gradients arriving one at a time in flat order reproduce the static
    bucket grid; a sync point launches the completed prefix early; a gradient
    out of order holds the frontier back; finish() covers the rest."""
    m = Transformer(model_config("tiny", **CFG)).build("cpu", seed=0)
    order = sorted(m.store.params, key=lambda p: p.offset)
    mb = 0.05
    dp, launched = _frontier_dp(m, mb, min_mb=0.001)
    for p in order:
        m.store.grad_ready(p)
    dp.finish()
    assert launched == [(b.start, b.end) for b in plan_buckets(m.store, int(mb * 2 ** 20))]

    dp, launched = _frontier_dp(m, 100.0, min_mb=0.001)  # buckets never fill
    half = len(order) // 2
    for p in order[1:half]:  # the first gradient is late
        m.store.grad_ready(p)
    m.store.grad_sync()
    assert launched == []  # nothing final from offset 0 yet
    m.store.grad_ready(order[0])
    m.store.grad_sync()
    assert launched == [(0, order[half].offset)]
    for p in order[half:]:
        m.store.grad_ready(p)
    dp.finish()
    assert launched[-1] == (order[half].offset, m.store.total)


def _cli(tmp, *sets, nproc=2):
    cmd = [sys.executable, "-m", "tensorflow_distributed_on_gke_amd", "train", "--config",
           os.path.join(ROOT, "configuration", "settings.yaml"), "--nproc", str(nproc),
           "--master-port", str(_free_port())]
    base = ["preset=tiny", "steps_per_epoch=6", "log_every=3", "local_batch_size=4", "src_len=10",
            "tgt_len=10", "src_vocab=300", "tgt_vocab=300", "snapshot_every_epochs=1",
            "validation_steps=1", "learning_rate=0.001", "worker_count=2", "check_replicas_every=2"]
    for kv in base + list(sets):
        cmd += ["--set", kv]
    env = dict(os.environ, PYTHONPATH=ROOT)
    env.pop("RANK", None)
    return subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True, timeout=300)


def test_train_cli_fault_injection_and_resume(tmp_path):
    """2 ranks; rank 1 dies mid epoch 2 -> launcher stops the job with its
    exit code; the restarted job resumes from the epoch-1 state and finishes."""
    r = _cli(tmp_path, "epochs=3", "kill_at_step=9")
    assert r.returncode == 17, r.stdout + r.stderr
    assert "Epoch 1 Loss" in r.stdout and "Epoch 2 Loss" not in r.stdout
    r = _cli(tmp_path, "epochs=3")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Resuming from" in r.stdout and "at epoch 2" in r.stdout
    assert "Epoch 1 Batch" not in r.stdout and "Epoch 3 Loss" in r.stdout
    assert "Time taken for 1 epoch" in r.stdout
    snaps = tmp_path / "snapshots" / "kubernetes-transformer-training"
    assert (snaps / "training-snapshots" / "initial_model" / "variables" / "variables.index").exists()
    assert (snaps / "training-snapshots_2" / "weights_snapshot_2" / "model_weights.index").exists()


def test_rank_dying_mid_backward_stops_the_job(tmp_path):
    """Failure detection: rank 1 exits inside step 4's backward, after some
    gradient all-reduce spans were launched, while rank 0 is blocked in the
    matching collective. The launcher must see the exit, stop rank 0 and exit
    with rank 1's code well within the process-group timeout -- no hang."""
    import time

    t0 = time.time()
    r = _cli(tmp_path, "epochs=2", "kill_at_step=4", "kill_point=backward", "kill_rank=1",
             "bucket_mb=0.02", "resume=false")
    dt = time.time() - t0
    # (rank 1's exit code 17, or rank 0's own failure if it surfaces first)
    assert r.returncode != 0, r.stdout + r.stderr
    assert "exiting in the backward of step 4" in r.stdout, r.stdout
    assert "Epoch 1 Loss" not in r.stdout  # died inside epoch 1 (6 steps)
    assert dt < 120, dt


def test_main_thread_collective_refused_while_spans_in_flight():
    """A main-thread collective (metrics, barrier, broadcast) issued while a
    gradient span is still in flight could interleave differently on
    different ranks: DataParallel refuses it, and a poisoned instance (a
    collective failed or was never issued) refuses everything."""
    m = Transformer(model_config("tiny", **CFG)).build("cpu", seed=0)
    dp = DataParallel(m.store, bucket_mb=100.0)
    dp.world = 2
    dp._outstanding = 1
    with pytest.raises(RuntimeError, match="not waited for"):
        dp.allreduce_metrics(torch.zeros(2))
    with pytest.raises(RuntimeError, match="not waited for"):
        dp.barrier()
    dp._outstanding = 0
    dp.poisoned = "test"
    with pytest.raises(RuntimeError, match="poisoned"):
        dp.check_quiescent("x")
    with pytest.raises(RuntimeError, match="poisoned"):
        dp.all_reduce_async(torch.zeros(4))


def test_segmented_capture_defers_collectives(monkeypatch):
    """While a step is captured as a segmented graph (train/graphs.py) the
    data-parallel code must not issue any collective: each all-reduce and the
    two tail wait points become recorded host calls, which issue / wait in
    order when replayed."""
    import torch.distributed as tdist

    m = Transformer(model_config("tiny", **CFG)).build("cpu", seed=0)
    order = sorted(m.store.params, key=lambda p: p.offset)
    dp = DataParallel(m.store, bucket_mb=0.05, min_mb=0.001)
    dp.active = True
    m.store.clear_grad_hooks()
    m.store.on_grad_ready(dp._on_ready)
    m.store.on_grad_sync(dp._on_sync)
    issued = []

    class _Work:
        def __init__(self, t):
            self.t, self.waited = t, False

        def wait(self):
            self.waited = True

    def fake_all_reduce(t, group=None, async_op=False):
        issued.append(_Work(t))
        return issued[-1]

    monkeypatch.setattr(tdist, "all_reduce", fake_all_reduce)

    class _Rec:
        def __init__(self):
            self.calls = []

        def cut(self, fn):
            self.calls.append(fn)

    rec = _Rec()
    dp.recorder = rec
    for p in order:
        m.store.grad_ready(p)
    dp.finish()
    dp.recorder = None
    spans = [(b.start, b.end) for b in dp.last_buckets]
    assert len(spans) > 2 and issued == []
    assert len(rec.calls) == len(spans) + 2  # one issue per span, two wait points
    for fn in rec.calls:  # "replay"
        fn()
    assert [(w.t.data_ptr() - m.store.flat_grad.data_ptr()) // 4 for w in issued] == [s for s, _ in spans]
    assert all(w.waited for w in issued)
    # eager (no recorder): issued immediately, waited in finish
    issued.clear()
    for p in order:
        m.store.grad_ready(p)
    assert len(issued) == len(spans) - 1  # the last span is launched by finish()
    dp.finish()
    assert len(issued) == len(spans) and all(w.waited for w in issued)
