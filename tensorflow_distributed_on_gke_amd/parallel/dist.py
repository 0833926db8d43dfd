"""Process-group bring-up: one process per GPU, torch.distributed over RCCL
(backend "nccl" is RCCL on ROCm) for GPU runs, gloo for CPU runs.

Rendezvous is env:// (MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE, as set by
`torch.distributed.run`, our local launcher, or the Kubernetes bootstrap in
cluster/k8s.py), replacing the reference's TF_CONFIG + gRPC bring-up
(reference: distributed_training_transformer/cluster/cluster.py:56-66).
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


# process-group timeout (seconds): a collective that does not complete within
# it aborts the process (RCCL async error handling) instead of hanging
PG_TIMEOUT_S = float(os.environ.get("TDG_DIST_TIMEOUT_S", "600"))


@dataclass
class DistInfo:
    rank: int
    world: int
    local_rank: int
    device: torch.device

    @property
    def chief(self) -> bool:
        """Rank 0 is the chief (reference: cluster.py:74-79)."""
        return self.rank == 0


def init_distributed(device: str = "auto", timeout_s: float = PG_TIMEOUT_S, force: bool = False) -> DistInfo:
    """`force`: create the process group even for a single rank (exercises the
    RCCL data-parallel path on one GPU)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_cuda = torch.cuda.is_available() if device == "auto" else device.startswith("cuda")
    if use_cuda:
        # (more ranks than GPUs only for rehearsals with TDG_DIST_BACKEND=gloo)
        dev = torch.device("cuda", local_rank % max(torch.cuda.device_count(), 1))
        torch.cuda.set_device(dev)
    else:
        dev = torch.device("cpu")
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        # RCCL async error handling: a dead peer aborts collectives instead of
        # hanging (failure detection; the reference relied on MWMS defaults).
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        # TDG_DIST_BACKEND=gloo: a multi-rank rehearsal of the GPU data-parallel
        # path on ONE GPU (RCCL needs a device per rank); production is RCCL
        backend = os.environ.get("TDG_DIST_BACKEND") or ("nccl" if use_cuda else "gloo")
        kw = dict(backend=backend, init_method="env://", rank=rank,
                  world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if use_cuda and backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(**kw)
    return DistInfo(rank, world, local_rank, dev)


def barrier() -> None:
    if dist.is_initialized():
        if torch.cuda.is_available() and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def shutdown() -> None:
    if dist.is_initialized():
        dist.destroy_process_group()
