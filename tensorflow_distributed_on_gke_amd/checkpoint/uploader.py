"""Snapshot uploader with unique folder naming and pluggable storage.

Reference behaviour (distributed_training_transformer/checkpoint.py:10-131,
__main__.py:139-169): the chief's first `take_snapshot` saves the whole model
to `<tmp>/model_uploader[_N]/initial_model` and uploads the directory to a
fresh unique folder under `<bucket>/<base folder>`; every later snapshot saves
weights into a fresh local `weights_snapshots/model_weights[_N]/model_weights`
prefix and uploads it to `<root>/weights_snapshot[_N]`.

Storage is pluggable: `LocalStorage` (a directory standing in for the bucket;
the default — GPU boxes have no network) or `GCSStorage` (Google Cloud Storage
through `google-cloud-storage`, only if that package is installed).

The reference's `initial_model` is a Keras SavedModel; without TensorFlow we
write the SavedModel variable layout (`initial_model/variables/variables.*`,
a TensorBundle) plus `model_config.json` instead of `saved_model.pb`.
"""
from __future__ import annotations

import json
import os
import shutil
from pathlib import Path
from typing import Optional

from tensorflow_distributed_on_gke_amd.checkpoint import bundle
from tensorflow_distributed_on_gke_amd.checkpoint.naming import new_directory_name, unique_name


class Storage:
    scheme = "storage"

    def exists(self, prefix: str) -> bool:
        raise NotImplementedError

    def upload_file(self, local: str, remote: str) -> None:
        raise NotImplementedError

    def describe(self, folder: str) -> str:
        raise NotImplementedError


class LocalStorage(Storage):
    """A local directory acting as the bucket."""

    def __init__(self, root: str):
        self.root = Path(root)
        self.root.mkdir(parents=True, exist_ok=True)

    def exists(self, prefix: str) -> bool:
        # GCS `list_blobs(prefix=..., max_results=1)` semantics: true if any
        # object's name starts with `prefix` (reference: checkpoint.py:120-131)
        for f in self.root.rglob("*"):
            if f.is_file() and str(f.relative_to(self.root)).startswith(prefix):
                return True
        return False

    def upload_file(self, local: str, remote: str) -> None:
        dst = self.root / remote
        dst.parent.mkdir(parents=True, exist_ok=True)
        shutil.copy2(local, dst)

    def describe(self, folder: str) -> str:
        return f"local storage {self.root}/{folder}"


class GCSStorage(Storage):  # pragma: no cover - needs network + google-cloud-storage
    def __init__(self, bucket: str, key_path: Optional[str] = None):
        try:
            from google.cloud import storage  # type: ignore
        except ImportError as e:
            raise RuntimeError("GCSStorage needs the google-cloud-storage package") from e
        client = (storage.Client.from_service_account_json(key_path) if key_path
                  else storage.Client())
        self.bucket_name = bucket
        self.client = client
        self.bucket = client.get_bucket(bucket)

    def exists(self, prefix: str) -> bool:
        for _ in self.client.list_blobs(self.bucket_name, max_results=1, prefix=prefix):
            return True
        return False

    def upload_file(self, local: str, remote: str) -> None:
        self.bucket.blob(remote).upload_from_filename(local)

    def describe(self, folder: str) -> str:
        return f"google cloud storage /{self.bucket_name}/{folder}"


def make_storage(bucket: str, key_path: Optional[str] = None, backend: str = "local",
                 local_root: str = "snapshots") -> Storage:
    if backend == "gcs":
        return GCSStorage(bucket, key_path)
    return LocalStorage(os.path.join(local_root, bucket))


def upload_directory(storage: Storage, local_directory: str, folder: str) -> None:
    root = Path(local_directory)
    for child in sorted(root.rglob("*")):
        if child.is_file():
            storage.upload_file(str(child), f"{folder}/{child.relative_to(root)}")


def safe_upload_directory(storage: Storage, local_directory: str, folder: str) -> str:
    new_folder = unique_name(folder, storage.exists)
    upload_directory(storage, local_directory, new_folder)
    return new_folder


def save_initial_model(model, directory: str) -> None:
    """SavedModel-layout stand-in: variables bundle + JSON model config."""
    os.makedirs(os.path.join(directory, "variables"), exist_ok=True)
    bundle.save_weights(model.store, os.path.join(directory, "variables", "variables"))
    with open(os.path.join(directory, "model_config.json"), "w") as f:
        json.dump({"class": "Transformer", "config": model.cfg.to_dict(),
                   "format": "tensorflow_distributed_on_gke_amd/initial_model/v1"}, f, indent=1)


class ModelUploader:
    def __init__(self, storage: Storage, base_folder: str, local_temporary_directory: str):
        self.storage = storage
        self.local_directory = new_directory_name(local_temporary_directory + "/model_uploader")
        os.makedirs(self.local_directory)
        self.cloud_base_folder_name = base_folder
        self.cloud_root_folder: Optional[str] = None
        self.last_upload_folder: Optional[str] = None

    def take_snapshot(self, model) -> None:
        if self.cloud_root_folder is None:
            save_initial_model(model, self.local_directory + "/initial_model")
            self.cloud_root_folder = safe_upload_directory(self.storage, self.local_directory,
                                                           self.cloud_base_folder_name)
            self.last_upload_folder = self.cloud_root_folder + "/initial_model"
        else:
            save_dir = new_directory_name(self.local_directory + "/weights_snapshots/model_weights")
            bundle.save_weights(model.store, save_dir + "/model_weights")
            self.last_upload_folder = safe_upload_directory(
                self.storage, save_dir, self.cloud_root_folder + "/weights_snapshot")

    def last_upload_location(self) -> str:
        return self.storage.describe(self.last_upload_folder or "")
