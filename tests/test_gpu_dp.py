"""The GPU data-parallel step with 2 ranks, rehearsed on ONE GPU: two
processes on cuda:0 exchange gradients over gloo (RCCL needs a device per
rank; the 8-GPU RCCL runs are the driver's). Everything else is the
production path: HIP kernels, deferred weight gradients launched in waves at
layer ends (a small wave forces problems to be cut across launches), the
frontier all-reduce spans, Adam. The update must match one process that runs
both ranks' batches with the reference's loss scaling (per-replica token mean
/ workers, SUM-reduced gradients), and the replicas must stay bitwise equal.
The "seg" cases run the step as the segmented HIP graph the multi-GPU bench
uses (train/graphs.py: graph segments with the collectives issued eagerly
between them), captured on the first batch and replayed on every step."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CFG = dict(d_model=512, heads=8, d_ff=2048, src_vocab=1000, tgt_vocab=1000, dropout=0.0)
STEPS = 3
ADAM = dict(lr=0.01, eps=1.0)


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(rank, i):
    g = torch.Generator().manual_seed(100 * i + rank)
    src = torch.randint(4, 1000, (8, 64), generator=g)
    tgt = torch.randint(4, 1000, (8, 65), generator=g)
    src[:, 50 + rank:] = 0
    tgt[:, 40 + 3 * rank:] = 0
    return src, tgt


def _worker(rank, world, port, out, opt_mode, loss_mode, graph, comm_thread="1", comm_bf16=False,
            signal="1"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), TDG_DIST_BACKEND="gloo",
                      TDG_DP_GRAPH=graph or "0", TDG_DP_COMM_THREAD=comm_thread, TDG_DP_SIGNAL=signal)
    from tensorflow_distributed_on_gke_amd.train import step as step_mod
    step_mod.WAVE_TILES = 37  # small waves: problems cut across launches
    step_mod.DP_OVERLAP_OPT = opt_mode
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.parallel import dist as tdist
    from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    kk.AUTOTUNE = False  # same GEMM configs as the reference process (bf16 rounding)
    info = tdist.init_distributed("cuda")
    m = Transformer(model_config("tiny", **CFG)).build(info.device, seed=1 + rank)
    opt = Adam(m.store, m.cfg.d_model, **ADAM)
    ddp = DataParallel(m.store, bucket_mb=1.0, comm_dtype=torch.bfloat16 if comm_bf16 else None)
    assert (ddp._thread is not None) == (comm_thread == "force")
    if ddp._thread is not None:  # issue points in a segmented graph: signal kernel or cut + event
        assert (ddp._thread.signal is not None) == (signal != "0")
    ddp.broadcast_params(0)
    step = TrainStep(m, opt, ddp, workers=world, seed=5, loss_mode=loss_mode)
    assert step.global_mean == (loss_mode == "global_mean")
    assert step.rt.wgrad is not None and step.rt.wgrad.wave_tiles == 37
    if graph:
        src, tgt = _batch(rank, 0)
        assert step.capture(src.to(info.device), tgt.to(info.device))  # trains nothing
        assert step.segments is not None and step.segments.num_calls >= 2
        assert opt.iterations == 0
        if ddp._thread is not None and signal != "0":
            # one signal per span, issue jobs handed over before their segment
            assert ddp._thread.signal.value() == 0
    losses = []
    for i in range(STEPS):
        src, tgt = _batch(rank, i)
        losses.append(step(src.to(info.device), tgt.to(info.device)).clone().cpu())
        ddp.verify_replicas()
    torch.cuda.synchronize()
    assert opt.iterations == STEPS
    if graph and ddp._thread is not None and signal != "0":
        # every handed-over issue job met its signal (one per span, plus the
        # global token count's all-reduce under global_mean)
        sig = ddp._thread.signal
        assert sig.value() == sig.expected >= STEPS * len(ddp.last_buckets)
    torch.save({"flat": m.store.flat.cpu(), "loss": torch.stack(losses), "nb": len(ddp.last_buckets)},
               f"{out}.{rank}")
    ddp.close()
    tdist.barrier()
    tdist.shutdown()


@pytest.mark.parametrize("world,opt_mode,loss_mode,graph,comm_thread,comm_bf16,signal", [
    (2, "0", "replica_mean", "", "0", False, "1"), (2, "tail", "replica_mean", "", "0", False, "1"),
    (2, "tail", "global_mean", "", "0", False, "1"), (2, "tail", "replica_mean", "seg", "0", False, "1"),
    (2, "0", "global_mean", "seg", "0", False, "1"),
    # the host comm thread (default on RCCL, TDG_DP_COMM_THREAD) driven over gloo
    (2, "tail", "replica_mean", "", "force", False, "1"), (2, "tail", "replica_mean", "seg", "force", False, "1"),
    (2, "tail", "global_mean", "seg", "force", False, "1"),
    # ... with the segmented graph cut at each issue point (event) instead of
    # the in-graph signal kernel (TDG_DP_SIGNAL=0)
    (2, "tail", "global_mean", "seg", "force", False, "0"),
    # four ranks on the production path: segmented graph, bf16 gradient
    # all-reduce, global token-mean loss -- with either issue path
    (4, "tail", "global_mean", "seg", "0", True, "1"), (4, "tail", "global_mean", "seg", "force", True, "1")])
def test_gpu_dp_rehearsal_matches_single_process(tmp_path, world, opt_mode, loss_mode, graph, comm_thread,
                                                 comm_bf16, signal, monkeypatch):
    from tensorflow_distributed_on_gke_amd.models.layers import RunCtx
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.train.optim import Adam

    out = str(tmp_path / "res")
    mp.start_processes(_worker, args=(world, _port(), out, opt_mode, loss_mode, graph, comm_thread, comm_bf16,
                                      signal),
                       nprocs=world, join=True, start_method="spawn")
    rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    r0 = rs[0]
    for r in rs[1:]:
        assert torch.equal(r0["flat"], r["flat"])  # replicas bitwise identical
    assert r0["nb"] > 2  # several spans launched from inside backward
    # single process: both batches, gradients accumulated, per-layer wgrad.
    # Autotuning off on both sides: the ranks and this process would otherwise
    # time-pick GEMM tiles independently, and a different summation order
    # flips bf16 roundings of intermediate gradients (~1e-2 relative drift)
    monkeypatch.setattr(kk, "AUTOTUNE", False)
    m = Transformer(model_config("tiny", **CFG)).build("cuda", seed=1)
    init = m.store.flat.clone()
    opt = Adam(m.store, m.cfg.d_model, **ADAM)
    losses = []
    for i in range(STEPS):
        # global token mean: both parts normalised by the global label count
        n_all = float(sum(int((_batch(r, i)[1][:, 1:] != 0).sum()) for r in range(world)))

        def fill(t, n=n_all):
            t.fill_(n)

        for r in range(world):
            rt = RunCtx(training=True, dropout=0.0, seed=5, store=m.store,
                        ctr=torch.zeros(1, dtype=torch.int64, device="cuda"), accumulate=r > 0)
            src, tgt = _batch(r, i)
            if loss_mode == "global_mean":
                o = m.loss_and_backward(src.cuda(), tgt.cuda(), rt, 1.0, ntok_sum=fill)
            else:
                o = m.loss_and_backward(src.cuda(), tgt.cuda(), rt, float(world))
            if r == 0:
                losses.append(o.clone().cpu())
        opt.apply()
    ref = m.store.flat.cpu()
    moved = (ref - init.cpu()).norm()
    assert moved > 0
    rel = (r0["flat"] - ref).norm() / moved
    print(f"world={world} opt_mode={opt_mode} bf16_comm={comm_bf16}: rel {rel:.3e}")
    # bf16 gradient all-reduce: the update matches to bf16 precision
    tol = 2e-2 if comm_bf16 else 1e-3
    assert rel < tol, f"DP update differs from the single-process update: rel {rel:.3e}"
    assert torch.allclose(r0["loss"], torch.stack(losses), rtol=1e-3, atol=1e-4)


def _fp8_worker(rank, world, port, out, graph, comm_thread="force"):
    """Config 5's data-parallel step (fp8 forward + FFN backward, per-bucket
    Adam at the tail, bf16 gradient all-reduce) with `world` ranks on cuda:0;
    collectives issued by the host comm thread (comm_thread "force": the path
    choose_dp_mode may pick on RCCL) or the process group's own handoff."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), TDG_DIST_BACKEND="gloo",
                      TDG_DP_GRAPH=graph or "0", TDG_DP_COMM_THREAD=comm_thread)
    from tensorflow_distributed_on_gke_amd.train import step as step_mod
    step_mod.WAVE_TILES = 37
    step_mod.DP_OVERLAP_OPT = "tail"
    from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
    from tensorflow_distributed_on_gke_amd.ops import fp8 as F
    from tensorflow_distributed_on_gke_amd.ops import kernels as kk
    from tensorflow_distributed_on_gke_amd.parallel import dist as tdist
    from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    from tensorflow_distributed_on_gke_amd.train.step import TrainStep

    kk.AUTOTUNE = False
    info = tdist.init_distributed("cuda")
    # hd 64 and sequences > 128: the e4m3 attention forward runs too
    cfg = model_config("tiny", d_model=128, heads=2, d_ff=512, src_vocab=1000, tgt_vocab=1000,
                       dropout=0.1)
    m = Transformer(cfg).build(info.device, seed=1 + rank)
    opt = Adam(m.store, m.cfg.d_model, lr=1e-3)
    ddp = DataParallel(m.store, bucket_mb=0.25, comm_dtype=torch.bfloat16)
    assert (ddp._thread is not None) == (comm_thread == "force")
    ddp.broadcast_params(0)
    st = F.Fp8State(m)  # after the broadcast: weight scales from the common weights
    st.weights.calibrate()
    step = TrainStep(m, opt, ddp, workers=world, seed=5, fp8_state=st, loss_mode="global_mean")
    assert ddp.opt is not None, "per-bucket Adam must be attached under fp8"
    g = torch.Generator().manual_seed(7 + rank)

    def batch():
        src = torch.randint(4, 1000, (4, 160), generator=g)
        tgt = torch.randint(4, 1000, (4, 161), generator=g)
        return src.to(info.device), tgt.to(info.device)

    if graph:
        assert step.capture(*batch())
        assert step.segments is not None
    losses = []
    for i in range(4):
        losses.append(float(step(*batch())[0]))
        ddp.verify_replicas()
    torch.cuda.synchronize()
    wslots = [i for i, n in enumerate(st.meta.names) if n.startswith(("w:", "wt:"))]
    torch.save({"flat": m.store.flat.cpu(), "wscale": st.meta.scale[wslots].cpu(),
                "w8": [w8.view(torch.uint8).cpu() for _, w8, _, _ in st.weights.items],
                "loss": losses}, f"{out}.{rank}")
    ddp.close()
    tdist.barrier()
    tdist.shutdown()


@pytest.mark.parametrize("world,graph,comm_thread", [(2, "seg", "force"), (4, "seg", "force"),
                                                     (2, "", "force"), (2, "seg", "0")])
def test_gpu_dp_fp8_replicas_identical(tmp_path, world, graph, comm_thread):
    """fp8 + data parallel (BASELINE config 5 is DP = 8): replicas stay
    bitwise equal, every rank derives the same weight scales and e4m3 weight
    copies, and the losses are finite."""
    out = str(tmp_path / "res")
    mp.start_processes(_fp8_worker, args=(world, _port(), out, graph, comm_thread), nprocs=world,
                       join=True, start_method="spawn")
    rs = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    for r in rs[1:]:
        assert torch.equal(rs[0]["flat"], r["flat"])
        assert torch.equal(rs[0]["wscale"], r["wscale"])
        for a, b in zip(rs[0]["w8"], r["w8"]):
            assert torch.equal(a, b)
    for r in rs:
        assert all(l == l and 0 < l < 20 for l in r["loss"]), r["loss"]


def test_gpu_rank_dying_mid_backward_with_comm_thread(tmp_path):
    """Failure detection on the GPU path: two ranks on one GPU (gloo), host
    comm thread forced on, eager steps; rank 1 exits inside a backward while
    rank 0's comm thread has spans queued or in flight. The launcher must
    stop rank 0 and exit with rank 1's code, quickly, with no hang."""
    import subprocess
    import sys
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "tensorflow_distributed_on_gke_amd", "train", "--config",
           os.path.join(root, "configuration", "settings.yaml"), "--nproc", "2", "--master-port", str(_port()),
           "--device", "cuda"]
    for kv in ["preset=tiny", "steps_per_epoch=6", "log_every=3", "local_batch_size=4", "src_len=16",
               "tgt_len=16", "src_vocab=300", "tgt_vocab=300", "snapshot_every_epochs=0",
               "validation_steps=1", "worker_count=2", "epochs=1", "hip_graph=false", "resume=false",
               "bucket_mb=0.02", "kill_at_step=3", "kill_point=backward", "kill_rank=1"]:
        cmd += ["--set", kv]
    env = dict(os.environ, PYTHONPATH=root, TDG_DIST_BACKEND="gloo", TDG_DP_COMM_THREAD="force")
    env.pop("RANK", None)
    t0 = time.time()
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    # either exit may be seen first: rank 1's injected one (17), or rank 0
    # failing its collective (the comm thread surfaces the peer loss)
    assert r.returncode != 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "exiting in the backward of step 3" in r.stdout
    assert "Epoch 1 Loss" not in r.stdout
    assert time.time() - t0 < 180
