import os

import pytest

from tensorflow_distributed_on_gke_amd.config import load_settings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_keys():
    s = load_settings(os.path.join(ROOT, "configuration", "settings.yaml"))
    assert s.local_batch_size == 64 and s.worker_count == 3
    assert s.cloud_storage_bucket_name == "kubernetes-transformer-training"
    assert s.cloud_storage_upload_folder == "training-snapshots"
    assert s.global_batch(3) == 192


def test_overrides_and_coercion():
    s = load_settings(None, ["epochs=3", "preset=tiny", "copy_task=false", "learning_rate=0.001",
                             "warm_start=saved/2/model_weights", "hip_graph=1", "learning_rate=None"])
    assert s.epochs == 3 and s.preset == "tiny" and s.copy_task is False
    assert s.warm_start == "saved/2/model_weights" and s.hip_graph is True and s.learning_rate is None


def test_unknown_keys(tmp_path):
    with pytest.raises(KeyError):
        load_settings(None, ["nope=1"])
    p = tmp_path / "s.yaml"
    p.write_text("local_batch_size: 8\nbogus: 1\n")
    with pytest.raises(KeyError):
        load_settings(str(p))
    with pytest.raises(ValueError):
        load_settings(None, ["epochs"])


def test_profiler_trace_written(tmp_path, monkeypatch):
    """profile_dir: a torch.profiler Chrome trace of the first steps (CPU here,
    roctracer HIP kernels on the GPU)."""
    from tensorflow_distributed_on_gke_amd.config import Settings
    from tensorflow_distributed_on_gke_amd.parallel.dist import DistInfo
    from tensorflow_distributed_on_gke_amd.train.loop import Trainer
    import torch

    monkeypatch.chdir(tmp_path)
    s = Settings(preset="tiny", local_batch_size=4, src_len=8, tgt_len=8, src_vocab=40, tgt_vocab=40,
                 epochs=1, steps_per_epoch=6, validation_steps=1, log_every=100,
                 snapshot_every_epochs=0, resume=False, profile_dir=str(tmp_path / "trace"),
                 profile_steps=2)
    Trainer(s, DistInfo(0, 1, 0, torch.device("cpu")), log=lambda m: None).fit()
    traces = list((tmp_path / "trace").glob("*.json"))
    assert traces and traces[0].stat().st_size > 0
