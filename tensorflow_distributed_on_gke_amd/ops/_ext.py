"""Loading of the native extensions.

`_C` holds the gfx950 HIP kernels; `_native` the host runtime (TensorBundle
I/O, CRC32C, data loader). Both are built in-tree by `_build.py`.

GPU ops never fall back to PyTorch: if `_C` is missing or was built for another
architecture, the first GPU op raises. CPU tensors take the plain-PyTorch
reference paths inside the layer ops (`models/layers.py`, e.g.
`_ref_attn_fwd`), used by the CPU test-suite and the tiny CPU config.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mods: dict = {}


def _load(name: str):
    with _lock:
        if name in _mods:
            return _mods[name]
        try:
            mod = importlib.import_module(f"tensorflow_distributed_on_gke_amd.{name}")
        except ImportError:
            if os.environ.get("TDG_NO_AUTOBUILD"):
                raise
            from tensorflow_distributed_on_gke_amd import _build

            _build.build()
            mod = importlib.import_module(f"tensorflow_distributed_on_gke_amd.{name}")
        _mods[name] = mod
        return mod


def C():
    """The HIP kernel module. Raises (never silently degrades) if unavailable."""
    import torch  # noqa: F401  (libtorch must be loaded first)

    try:
        return _load("_C")
    except Exception as e:  # pragma: no cover - exercised only on broken installs
        raise RuntimeError(
            "tensorflow_distributed_on_gke_amd: the gfx950 HIP extension `_C` is not "
            "available; run `python -m tensorflow_distributed_on_gke_amd._build`"
        ) from e


def native():
    return _load("_native")
