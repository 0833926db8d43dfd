"""Run configuration.

The YAML file keeps the reference's four keys
(reference: configuration/settings.yaml:1-4, read at distributed_training_transformer/__main__.py:20-25):
`local_batch_size`, `worker_count`, `cloud_storage_bucket_name`,
`cloud_storage_upload_folder`. Everything the reference hard-codes
(__main__.py:39-43, 56-73, 89, 139-169) becomes an optional key with the
reference value as default, and any key can be overridden on the command line
with `--set key=value`.

Divergence (fixes a reference bug): the data-parallel world
size comes from the runtime (WORLD_SIZE / the cluster), not from
`worker_count`; `worker_count` is only the expected size, checked at start-up.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import yaml


@dataclass
class Settings:
    # --- the reference's four keys
    local_batch_size: int = 64
    worker_count: int = 1
    cloud_storage_bucket_name: str = "kubernetes-transformer-training"
    cloud_storage_upload_folder: str = "training-snapshots"
    # --- model (reference __main__.py:39-43 -> preset "reference")
    preset: str = "reference"
    layers: Optional[int] = None
    d_model: Optional[int] = None
    heads: Optional[int] = None
    d_ff: Optional[int] = None
    dropout: float = 0.1
    label_smoothing: float = 0.0
    src_vocab: int = 7765
    tgt_vocab: int = 7010
    max_len: int = 1000
    # --- optimisation (reference __main__.py:56-73)
    warmup_steps: int = 4000
    beta1: float = 0.9
    beta2: float = 0.98
    epsilon: float = 1e-9
    learning_rate: Optional[float] = None  # None -> Noam schedule
    # --- loop (reference __main__.py:89, 149-180)
    epochs: int = 20
    steps_per_epoch: int = 200
    validation_steps: int = 20
    log_every: int = 50
    snapshot_every_epochs: int = 5
    # --- data: "synthetic" token pairs, or "text": TSV source<TAB>target files
    # (data/text.py, the reference's TED pipeline on local files; an epoch is
    # one pass over train_file, steps_per_epoch / validation_steps ignored)
    data: str = "synthetic"
    train_file: Optional[str] = None
    validation_file: Optional[str] = None
    src_tokenizer: Optional[str] = None  # WordPiece JSON; None: trained on train_file
    tgt_tokenizer: Optional[str] = None
    shuffle_buffer: int = 20000
    src_len: int = 40
    tgt_len: int = 40
    min_len: int = 4
    copy_task: bool = True
    seed: int = 0
    # --- checkpoint / storage (reference checkpoint.py, __main__.py:30,139-147)
    storage_backend: str = "local"
    storage_root: str = "snapshots"
    google_cloud_access_key_path: str = "configuration/gcp-access-key.json"
    temporary_directory: str = "temporary"
    warm_start: Optional[str] = None  # reference always loads saved_weights/2/model_weights
    resume: bool = True  # extension: resume from the newest local snapshot
    # --- runtime
    dtype: str = "bf16"
    bucket_mb: float = 64.0
    grad_comm_dtype: str = "fp32"  # fp32 | bf16 (gradient all-reduce payload)
    hip_graph: bool = False
    # variable-length (text) batches under hip_graph: each batch's source and
    # target-input lengths are padded up to a multiple of graph_bucket (capped
    # at max_len; semantically neutral -- attention, loss and LayerNorm are
    # length-masked) and one captured step per (source, target) bucket is kept,
    # at most graph_cache of them (least recently used evicted)
    graph_bucket: int = 32
    graph_cache: int = 64
    idle_after_train: bool = False  # reference __main__.py:183-186 keeps the pod alive
    check_replicas_every: int = 0  # debug: assert bitwise-identical replicas every N steps
    metrics_file: Optional[str] = None  # JSONL metrics sink (rank 0)
    profile_dir: Optional[str] = None  # torch.profiler (roctracer) Chrome trace of the first steps
    profile_steps: int = 5  # active profiled steps (after 1 wait + 1 warm-up step)
    kill_at_step: int = -1  # fault injection (tests): global step at which to exit
    kill_rank: int = -1  # rank that exits (-1: the last rank)
    # "step": exit after the step; "backward": exit in the middle of that
    # step's backward, once half of the gradients are final (peers are then
    # blocked inside a gradient all-reduce; eager steps only -- a captured
    # step runs no Python callbacks)
    kill_point: str = "step"
    # "replica_mean": the reference's per-replica token mean / workers
    # (transformer_model.py:11-17); "global_mean": sum of all replicas' token
    # losses / all replicas' label count (equal to the single-process loss on
    # the global batch, whatever the per-replica token counts)
    loss_mode: str = "replica_mean"

    def global_batch(self, world: int) -> int:
        return self.local_batch_size * world


def _coerce(cur: Any, value: str, ftype) -> Any:
    if value in ("None", "null") and "Optional" in str(ftype):
        return None
    if isinstance(cur, bool) or ftype in (bool, "bool", Optional[bool]):
        return str(value).lower() in ("1", "true", "yes", "on")
    for t in (int, float):
        if isinstance(cur, t) and not isinstance(cur, bool):
            return t(value)
    if value in ("None", "null", ""):
        return None
    try:
        return int(value)
    except ValueError:
        try:
            return float(value)
        except ValueError:
            return value


def load_settings(path: Optional[str] = None, overrides: Optional[List[str]] = None) -> Settings:
    s = Settings()
    names = {f.name: f for f in dataclasses.fields(Settings)}
    if path:
        with open(path) as f:
            data: Dict[str, Any] = yaml.safe_load(f) or {}
        unknown = set(data) - set(names)
        if unknown:
            raise KeyError(f"unknown settings keys: {sorted(unknown)}")
        for k, v in data.items():
            setattr(s, k, v)
    for ov in overrides or []:
        if "=" not in ov:
            raise ValueError(f"--set expects key=value, got {ov!r}")
        k, v = ov.split("=", 1)
        if k not in names:
            raise KeyError(f"unknown setting {k!r}")
        setattr(s, k, _coerce(getattr(s, k), v, names[k].type))
    return s
