#!/usr/bin/env python3
"""Headline benchmark: whole-node training tokens/sec of Transformer-base
(6 layers, d_model 512, 8 heads, d_ff 2048, vocab pt 7765 / en 7010) on
synthetic (source, target) pairs of length 128, bf16 compute, synchronous data
parallelism over RCCL on N MI355X GPUs (one process per GPU).

    python bench.py --gpus N --steps K --warmup W
    (N > 1: starts its own N ranks, one per GPU, when no launcher set
    WORLD_SIZE; under python -m torch.distributed.run --nproc-per-node N it
    is one of the N ranks. A world that is not N exits non-zero.)

A timed step is the full training step: forward, masked cross-entropy,
backward, bucketed gradient all-reduce, Adam update. Weak scaling: the local
batch (default 64 sentence pairs per GPU, the reference's local_batch_size,
configuration/settings.yaml) is fixed, so the global batch is 64*N.
tokens/step = global_batch * (src_len + tgt_len) = 64*N*256.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

# RCCL / HIP IPC between the ranks' processes needs the dmabuf IPC mode on
# these hosts (the legacy mode fails in hipIpcGetMemHandle); set before the
# first HIP call, for this process and the ranks it may launch
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config  # noqa: E402
from tensorflow_distributed_on_gke_amd.parallel import dist as tdist  # noqa: E402
from tensorflow_distributed_on_gke_amd.parallel.ddp import DataParallel  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.optim import Adam  # noqa: E402
from tensorflow_distributed_on_gke_amd.train.step import TrainStep  # noqa: E402
from tensorflow_distributed_on_gke_amd.data.synthetic import SyntheticPairs  # noqa: E402

METRIC = "tokens/sec (whole node), Transformer-base en-pt at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no number


def visible_gpus() -> int:
    """GPUs this process could use, counted WITHOUT initialising HIP (the
    launcher parent must not touch the GPU): the visible-devices lists if set,
    else the GPU nodes of the KFD topology (nodes with SIMDs)."""
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() and x.strip() != "-1"])
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(base)
    except OSError:
        return 0
    for node in nodes:
        try:
            with open(os.path.join(base, node, "properties")) as f:
                for line in f:
                    k, _, val = line.partition(" ")
                    if k == "simd_count" and int(val) > 0:
                        n += 1
                        break
        except (OSError, ValueError):
            continue
    return n


def self_launch(n: int) -> int:
    """Spawn `n` ranks of this script (one per GPU) and return their exit code.

    Runs BEFORE anything touches the GPU in this parent: children are plain
    subprocesses (never exec), each binds GPU LOCAL_RANK; the first child to
    fail takes the others down (cluster/launch.py). Counting devices does not
    initialise HIP. With fewer GPUs than ranks the request is refused (exit 2)
    unless TDG_DIST_BACKEND=gloo asks for a one-GPU rehearsal; on a host with
    no GPU the ranks run the CPU reference ops over gloo.
    """
    import socket

    from tensorflow_distributed_on_gke_amd.cluster import launch, rendezvous

    ngpu = visible_gpus()
    if 0 < ngpu < n and os.environ.get("TDG_DIST_BACKEND") != "gloo":
        print(f"bench.py: --gpus {n} requested but only {ngpu} GPU(s) are visible; refusing to "
              f"measure fewer ranks (set TDG_DIST_BACKEND=gloo for a shared-GPU rehearsal)",
              file=sys.stderr, flush=True)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    spec = rendezvous.ClusterSpec(0, 1, ["127.0.0.1"], "127.0.0.1", port)
    # the parent never initialises HIP: the ranks are fresh child processes
    # that each bind their own GPU
    assert not torch.cuda.is_initialized(), "bench.py launcher must not initialise HIP"
    extra = {}
    if 0 < ngpu < n and "GPU_MAX_HW_QUEUES" not in os.environ:
        # several ranks share a card (gloo rehearsal): one hardware queue each,
        # so the ranks' queues together stay within the card's queue slots (an
        # 8-rank rehearsal with 4 queues per rank aborted once inside a PyTorch
        # kernel with an illegal-instruction error; with 1 it ran clean)
        extra["GPU_MAX_HW_QUEUES"] = "1"
    return launch.launch([os.path.abspath(__file__)] + sys.argv[1:], n, spec, env_extra=extra)


def _fp8_precision() -> str:
    from tensorflow_distributed_on_gke_amd.ops.fp8 import precision_string
    return precision_string()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--preset", default="base")
    ap.add_argument("--local-batch", type=int, default=64)
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    ap.add_argument("--grad-comm", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce dtype (bf16 halves xGMI bytes)")
    ap.add_argument("--graph", type=int, default=-1,
                    help="1: capture the step in HIP graphs (default on for GPUs; data parallel: segmented graph)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--defer-wgrad", type=int, default=-1,
                    help="1: group weight gradients at the end of backward (default: on for 1 GPU)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                    help="fp8 (BASELINE config 5): every encoder/decoder projection GEMM in fp8 "
                         "(forward e4m3 x e4m3; dgrads and weight gradients e5m2 x e4m3), the "
                         "attention forward in e4m3, delayed per-tensor scaling; the per-op map "
                         "(ops/fp8.py precision_map) is printed in the record's dtype field")
    ap.add_argument("--save-tuned", default=None, help="write the autotuned GEMM table (JSON) here")
    ap.add_argument("--force-dp", type=int, default=0,
                    help="1: run the RCCL data-parallel path even with one rank (testing)")
    ap.add_argument("--verify-replicas", type=int, default=0,
                    help="1: after the timed steps (outside the timing), check that every rank's "
                         "weights are bitwise equal (DataParallel.verify_replicas; exits non-zero if not)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # `python bench.py --gpus N` with no launcher: start the N ranks here
        sys.exit(self_launch(args.gpus))

    info = tdist.init_distributed(force=bool(args.force_dp))
    world = info.world
    if world != args.gpus:
        # never print a one-GPU number under an N-GPU request
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks",
              file=sys.stderr, flush=True)
        tdist.shutdown()
        sys.exit(3)
    dev = info.device
    cfg = model_config(args.preset, max_src_len=max(1000, args.seq_len), max_tgt_len=max(1000, args.seq_len))
    model = Transformer(cfg).build(dev, seed=args.seed)
    opt = Adam(model.store, cfg.d_model)
    comm = torch.bfloat16 if args.grad_comm == "bf16" else None
    ddp = DataParallel(model.store, bucket_mb=args.bucket_mb, comm_dtype=comm,
                       force=bool(args.force_dp)) if (world > 1 or args.force_dp) else None
    if ddp is not None:
        ddp.broadcast_params(0)
    fp8_state = None
    if args.dtype == "fp8":
        from tensorflow_distributed_on_gke_amd.ops.fp8 import Fp8State
        fp8_state = Fp8State(model)
    step = TrainStep(model, opt, ddp, workers=world, seed=args.seed + 17, fp8_state=fp8_state,
                     defer_wgrad=None if args.defer_wgrad < 0 else bool(args.defer_wgrad))

    S = T = args.seq_len
    data = SyntheticPairs(batch=args.local_batch, src_len=S, tgt_len=T + 1, src_vocab=cfg.src_vocab,
                          tgt_vocab=cfg.tgt_vocab, seed=args.seed, rank=info.rank, world=world, pin=True)
    # pre-stage a few device batches so the timed loop measures the step
    batches = []
    for i in range(4):
        s, t = data.batch(i)
        batches.append((s.to(dev, non_blocking=True), t.to(dev, non_blocking=True)))

    # HIP graph by default. One GPU: the whole step is one graph. Data
    # parallel: a chain of graphs cut at the RCCL collectives, which stay
    # eager calls between the segments (train/graphs.py; TDG_DP_GRAPH=0 runs
    # the step eagerly)
    use_graph = args.graph if args.graph >= 0 else int(dev.type == "cuda")
    dp_select = None
    if use_graph and ddp is not None and ddp.active:
        # segmented graph or eager step, whichever measures faster on this node
        # (every rank takes the same decision; train.step.DP_AUTOSELECT = False: graph)
        dp_select = step.choose_dp_mode(*batches[0])
        use_graph = int(step.captured)
    elif use_graph:
        use_graph = int(step.capture(*batches[0]))
    for i in range(args.warmup):
        step(*batches[i % len(batches)])

    if dev.type == "cuda":
        torch.cuda.synchronize()
    tdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(*batches[i % len(batches)])
    if dev.type == "cuda":
        torch.cuda.synchronize()
    tdist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    if ddp is not None:
        # every rank reports its own decision and spans (they must agree)
        spans = [round((b.end - b.start) * 4 / 2 ** 20, 1) for b in ddp.last_buckets]
        print(f"[rank {info.rank}/{world}] dp_mode_select={dp_select} comm_issue={ddp.comm_choice} "
              f"all-reduce spans per step (MB, launch order): {spans}", file=sys.stderr, flush=True)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    verified = None
    if args.verify_replicas and ddp is not None and world > 1:
        ddp.verify_replicas()  # raises on divergence
        verified = True
    ms = elapsed / args.steps * 1000.0
    global_batch = args.local_batch * world
    tokens = global_batch * (S + T) * args.steps
    value = tokens / elapsed
    loss = float(step.last[0].item()) * world if dev.type == "cuda" else float(step.last[0])
    if info.rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": ("fp32 (CPU reference ops)" if dev.type != "cuda" else "bf16") if args.dtype == "bf16" else
                     _fp8_precision(),
            "data": f"synthetic (random-init weights, synthetic pt/en token pairs, full-length {S})",
            "config": {
                "model": f"transformer-{args.preset} ({cfg.layers}L, d_model={cfg.d_model}, "
                         f"heads={cfg.heads}, d_ff={cfg.d_ff}, vocab {cfg.src_vocab}/{cfg.tgt_vocab})",
                "global_batch": global_batch,
                "local_batch": args.local_batch,
                "seq_len": S,
                "parallelism": f"dp{world}",
                "hip_graph": (("segmented" if step.segments is not None else "single")
                              if use_graph else False),
                **({"dp_mode_select": dp_select} if dp_select else {}),
                **({"comm_issue": ddp.comm_choice} if ddp is not None else {}),
                "grad_comm": args.grad_comm,
                "defer_wgrad": step.rt.wgrad is not None,
                "bucket_mb": args.bucket_mb,
                "last_loss": round(loss, 4),
                **({"replicas_verified": verified} if verified is not None else {}),
            },
        }), flush=True)
    if args.save_tuned and info.rank == 0:
        from tensorflow_distributed_on_gke_amd.ops import kernels as _kk
        _kk.save_tuned(args.save_tuned)
    if ddp is not None:
        ddp.close()
    tdist.shutdown()


if __name__ == "__main__":
    main()
