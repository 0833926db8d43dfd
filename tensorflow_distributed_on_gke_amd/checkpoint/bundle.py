"""TensorFlow-compatible weight checkpoints (TensorBundle), without TensorFlow.

Writes / reads exactly what the reference's Keras `model.save_weights(prefix)`
produces and `load_weights(prefix)` consumes
(reference: distributed_training_transformer/checkpoint.py:75-88,
__main__.py:87, saved_weights/{1,2}/; format decoded in SURVEY.md §2.6):

  <prefix>.index                  SSTable of BundleEntryProto (native C++ writer:
                                  byte-identical to TF's for the same entries)
  <prefix>.data-00000-of-00001    raw little-endian f32 tensors, TF creation order
  checkpoint                      CheckpointState text file

Keys are the reference's object-path keys
(`encoder/encoder_layers/0/mha/query_generator_weights/kernel/.ATTRIBUTES/VARIABLE_VALUE`, ...)
and Dense kernels are stored in TF's [in, out] layout; the mapping to our fused
[out, in] parameters is carried by each Param's TFSlots.

The `_CHECKPOINTABLE_OBJECT_GRAPH` entry is synthesised from the key paths (a
TrackableObjectGraph with one node per path component); the reference's own
object-graph bytes live in the data blob it does not ship, so that entry is
not byte-verified (documented divergence).

Extension over the reference: `save_training_state` writes a second bundle with
the Adam slots and the iteration counter so training can resume exactly.
"""
from __future__ import annotations

import os
import re
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from tensorflow_distributed_on_gke_amd.models.params import ParamStore
from tensorflow_distributed_on_gke_amd.ops._ext import native

DT_FLOAT = 1
DT_INT64 = 9
OBJECT_GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"
SUFFIX = "/.ATTRIBUTES/VARIABLE_VALUE"


# ------------------------------------------------------------------ key order
_LN_RE = re.compile(r"^(encoder|decoder)/(?:encoder|decoder)_layers/(\d+)/layernorm(\d)/(gamma|beta)")
_LAYER_RE = re.compile(r"^(encoder|decoder)/(?:encoder|decoder)_layers/(\d+)/(mha|mha1|mha2|ffn)/(\S+?)/(kernel|bias)")
_SUB = {"mha": 0, "mha1": 0, "mha2": 1, "ffn": 2}
_DENSE = {"query_generator_weights": 0, "key_generator_weights": 1, "value_generator_weights": 2,
          "dense": 3, "layer_with_weights-0": 0, "layer_with_weights-1": 1}


def tf_creation_order(key: str) -> Tuple:
    """Sort key reproducing the reference data-file tensor order (Keras
    variable creation order): final layer, embeddings, all LayerNorms, then
    per layer q, k, v, dense (kernel, bias) and the FFN."""
    k = key[: -len(SUFFIX)] if key.endswith(SUFFIX) else key
    if k.startswith("final_layer/"):
        return (0, 0 if k.endswith("kernel") else 1)
    if k == "encoder/embedding/embeddings":
        return (1,)
    if k == "decoder/embedding/embeddings":
        return (2,)
    m = _LN_RE.match(k)
    if m:
        return (3, 0 if m.group(1) == "encoder" else 1, int(m.group(2)), int(m.group(3)),
                0 if m.group(4) == "gamma" else 1)
    m = _LAYER_RE.match(k)
    if m:
        return (4, 0 if m.group(1) == "encoder" else 1, int(m.group(2)), _SUB[m.group(3)],
                _DENSE.get(m.group(4), 9), 0 if m.group(5) == "kernel" else 1)
    return (5, k)


# ------------------------------------------------------------------ object graph
def _pb_varint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def _pb_field(num: int, wire: int, payload: bytes) -> bytes:
    return _pb_varint((num << 3) | wire) + payload


def _pb_bytes(num: int, b: bytes) -> bytes:
    return _pb_field(num, 2, _pb_varint(len(b)) + b)


def object_graph(keys: List[str]) -> bytes:
    """TrackableObjectGraph: root -> path components -> variable nodes whose
    attribute VARIABLE_VALUE points at the checkpoint key."""
    nodes: List[dict] = [{"children": [], "attr": None}]
    index: Dict[Tuple[int, str], int] = {}
    for key in sorted(k for k in keys if k.endswith(SUFFIX)):
        path = key[: -len(SUFFIX)].split("/")
        cur = 0
        for comp in path:
            nid = index.get((cur, comp))
            if nid is None:
                nid = len(nodes)
                nodes.append({"children": [], "attr": None})
                nodes[cur]["children"].append((nid, comp))
                index[(cur, comp)] = nid
            cur = nid
        nodes[cur]["attr"] = ("VARIABLE_VALUE", "/".join(path), key)
    out = bytearray()
    for n in nodes:
        body = bytearray()
        for nid, name in n["children"]:
            body += _pb_bytes(1, _pb_field(1, 0, _pb_varint(nid)) + _pb_bytes(2, name.encode()))
        if n["attr"] is not None:
            name, full, ckey = n["attr"]
            body += _pb_bytes(2, _pb_bytes(1, name.encode()) + _pb_bytes(2, full.encode()) +
                              _pb_bytes(3, ckey.encode()))
        out += _pb_bytes(1, bytes(body))
    return bytes(out)


# ------------------------------------------------------------------ tensors <-> TF layout
def tf_tensors(store: ParamStore) -> Dict[str, np.ndarray]:
    """{tf key: f32 numpy array in TF layout} from the f32 masters."""
    host = store.flat.detach().float().cpu()
    out = {}
    for p in store.params:
        full = host[p.offset: p.offset + p.numel].view(p.shape)
        for s in p.tf:
            t = full[s.row0: s.row1]
            if s.transpose:
                t = t.t()
            out[s.key] = np.ascontiguousarray(t.numpy(), dtype=np.float32)
    return out


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray], order=tf_creation_order,
                 with_object_graph: bool = True, state_file: bool = True) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    w = native().BundleWriter(prefix)
    for key in sorted(tensors, key=order):
        a = np.ascontiguousarray(tensors[key])
        dt = {np.dtype(np.float32): DT_FLOAT, np.dtype(np.int64): DT_INT64}[a.dtype]
        w.add(key, dt, list(a.shape), a.reshape(-1).view(np.uint8))
    if with_object_graph:
        w.add_string(OBJECT_GRAPH_KEY, object_graph(list(tensors)))
    w.finish()
    if not state_file:
        return
    state = os.path.join(os.path.dirname(os.path.abspath(prefix)), "checkpoint")
    base = os.path.basename(prefix)
    with open(state, "w") as f:
        f.write(f'model_checkpoint_path: "{base}"\nall_model_checkpoint_paths: "{base}"\n')


def read_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    r = native().BundleReader(prefix, verify)
    out = {}
    for key in r.keys():
        e = r.entry(key)
        if key == OBJECT_GRAPH_KEY or e["dtype"] not in (DT_FLOAT, DT_INT64):
            continue
        dt = np.float32 if e["dtype"] == DT_FLOAT else np.int64
        out[key] = np.frombuffer(r.read(key, verify), dtype=dt).reshape(e["shape"]).copy()
    return out


def bundle_entries(prefix: str) -> Dict[str, dict]:
    r = native().BundleReader(prefix, False)
    return {k: r.entry(k) for k in r.keys()}


def resolve_prefix(path: str) -> str:
    """Accept a directory holding a `checkpoint` state file, or a prefix."""
    if os.path.isdir(path):
        state = os.path.join(path, "checkpoint")
        if os.path.exists(state):
            m = re.search(r'model_checkpoint_path:\s*"([^"]+)"', open(state).read())
            if m:
                p = m.group(1)
                return p if os.path.isabs(p) else os.path.join(path, p)
        return os.path.join(path, "model_weights")
    return path


# ------------------------------------------------------------------ model-level API
def save_weights(store: ParamStore, prefix: str) -> None:
    """Keras `model.save_weights(prefix)` equivalent."""
    write_bundle(prefix, tf_tensors(store))


def load_weights(store: ParamStore, prefix: str, strict: bool = True) -> List[str]:
    """Keras `model.load_weights(prefix)` equivalent. Returns missing keys."""
    tensors = read_bundle(resolve_prefix(prefix))
    host = store.flat.detach().float().cpu().clone()
    missing = []
    for p in store.params:
        full = host[p.offset: p.offset + p.numel].view(p.shape)
        for s in p.tf:
            a = tensors.get(s.key)
            if a is None:
                missing.append(s.key)
                continue
            t = torch.from_numpy(a)
            if s.transpose:
                t = t.t()
            if tuple(t.shape) != tuple(full[s.row0: s.row1].shape):
                raise ValueError(f"{s.key}: checkpoint shape {tuple(a.shape)} does not match model")
            full[s.row0: s.row1].copy_(t)
    if strict and missing:
        raise KeyError(f"checkpoint {prefix} lacks {len(missing)} variables, e.g. {missing[:3]}")
    store.flat.copy_(host.to(store.flat.device))
    store.refresh_compute()
    return missing


def save_training_state(store: ParamStore, opt, prefix: str, extra: Optional[Dict[str, int]] = None) -> None:
    """Adam slots (m, v per variable, TF layout, Keras slot-style names) and
    the iteration counter -> `<prefix>_optimizer` bundle (resume extension)."""
    m = opt.m.detach().float().cpu()
    v = opt.v.detach().float().cpu()
    out: Dict[str, np.ndarray] = {}
    for p in store.params:
        for name, buf in (("m", m), ("v", v)):
            full = buf[p.offset: p.offset + p.numel].view(p.shape)
            for s in p.tf:
                t = full[s.row0: s.row1]
                if s.transpose:
                    t = t.t()
                out[s.key.replace(SUFFIX, f"/.OPTIMIZER_SLOT/optimizer/{name}/.ATTRIBUTES/VARIABLE_VALUE")] = \
                    np.ascontiguousarray(t.numpy())
    out["optimizer/iter/.ATTRIBUTES/VARIABLE_VALUE"] = np.array(opt.iterations, dtype=np.int64)
    for k, val in (extra or {}).items():
        out[f"training_state/{k}"] = np.array(int(val), dtype=np.int64)
    write_bundle(prefix + "_optimizer", out, order=lambda k: k, with_object_graph=False,
                 state_file=False)


def load_training_state(store: ParamStore, opt, prefix: str) -> Dict[str, int]:
    tensors = read_bundle(prefix + "_optimizer")
    m = opt.m.detach().float().cpu().clone()
    v = opt.v.detach().float().cpu().clone()
    for p in store.params:
        for name, buf in (("m", m), ("v", v)):
            full = buf[p.offset: p.offset + p.numel].view(p.shape)
            for s in p.tf:
                a = tensors[s.key.replace(SUFFIX, f"/.OPTIMIZER_SLOT/optimizer/{name}/.ATTRIBUTES/VARIABLE_VALUE")]
                t = torch.from_numpy(a)
                full[s.row0: s.row1].copy_(t.t() if s.transpose else t)
    opt.m.copy_(m.to(opt.m.device))
    opt.v.copy_(v.to(opt.v.device))
    opt.step.fill_(int(tensors["optimizer/iter/.ATTRIBUTES/VARIABLE_VALUE"].item()))
    return {k[len("training_state/"):]: int(a.item()) for k, a in tensors.items()
            if k.startswith("training_state/")}
