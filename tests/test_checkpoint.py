"""TensorBundle golden tests against the reference's shipped index files."""
import os

import numpy as np
import pytest
import torch

from tensorflow_distributed_on_gke_amd.checkpoint import bundle
from tensorflow_distributed_on_gke_amd.checkpoint.naming import new_directory_name, unique_name
from tensorflow_distributed_on_gke_amd.checkpoint.uploader import LocalStorage, ModelUploader
from tensorflow_distributed_on_gke_amd.models.transformer import Transformer, model_config
from tensorflow_distributed_on_gke_amd.ops._ext import native

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def _ref_index(n=2):
    return open(os.path.join(FIX, f"ref{n}_model_weights.index"), "rb").read()


@pytest.mark.parametrize("n", [1, 2])
def test_parse_reference_index(n):
    kv = native().parse_sstable(_ref_index(n), True)
    assert len(kv) == 174
    keys = [k.decode() for k, _ in kv]
    assert keys[0] == "" and keys[1] == "_CHECKPOINTABLE_OBJECT_GRAPH"
    assert keys == sorted(keys)
    ents = {k.decode(): native().decode_entry(v) for k, v in kv[1:]}
    fl = ents["final_layer/kernel/.ATTRIBUTES/VARIABLE_VALUE"]
    assert fl["shape"] == [128, 7010] and fl["offset"] == 0 and fl["size"] == 128 * 7010 * 4
    assert ents["encoder/embedding/embeddings/.ATTRIBUTES/VARIABLE_VALUE"]["shape"] == [7765, 128]
    assert ents["_CHECKPOINTABLE_OBJECT_GRAPH"]["dtype"] == 7
    total = sum(e["size"] for k, e in ents.items() if k != "_CHECKPOINTABLE_OBJECT_GRAPH")
    assert total == 4646882 * 4


def test_reference_index_rebuilt_byte_identical():
    data = _ref_index(2)
    n = native()
    kv = n.parse_sstable(data, True)
    assert all(n.encode_entry(n.decode_entry(v)) == v for _, v in kv[1:])
    assert kv[0][1] == n.encode_header(1, 1)
    assert n.build_sstable(kv) == data


def test_model_keys_and_shapes_match_reference():
    n = native()
    ref = {k.decode(): n.decode_entry(v) for k, v in n.parse_sstable(_ref_index(2), True)[1:]}
    m = Transformer(model_config("reference")).build("cpu", seed=0)
    ours = bundle.tf_tensors(m.store)
    assert set(ours) == set(ref) - {"_CHECKPOINTABLE_OBJECT_GRAPH"}
    for k, a in ours.items():
        assert list(a.shape) == ref[k]["shape"], k


def test_data_file_order_and_offsets_match_reference(tmp_path):
    n = native()
    ref = {k.decode(): n.decode_entry(v) for k, v in n.parse_sstable(_ref_index(2), True)[1:]}
    m = Transformer(model_config("reference")).build("cpu", seed=0)
    prefix = str(tmp_path / "model_weights")
    bundle.save_weights(m.store, prefix)
    ours = bundle.bundle_entries(prefix)
    for k, e in ref.items():
        if k == "_CHECKPOINTABLE_OBJECT_GRAPH":
            assert ours[k]["offset"] == e["offset"]  # object graph follows the 172 tensors
            continue
        assert ours[k]["offset"] == e["offset"] and ours[k]["size"] == e["size"], k
    assert open(tmp_path / "checkpoint").read().startswith('model_checkpoint_path: "model_weights"')


def test_roundtrip_bit_exact_and_crc(tmp_path):
    cfg = model_config("tiny", src_vocab=50, tgt_vocab=40)
    a = Transformer(cfg).build("cpu", seed=1)
    b = Transformer(cfg).build("cpu", seed=2)
    prefix = str(tmp_path / "w" / "model_weights")
    bundle.save_weights(a.store, prefix)
    bundle.load_weights(b.store, str(tmp_path / "w"))
    assert torch.equal(a.store.flat, b.store.flat)
    # corrupt one byte of the data file -> CRC failure
    data = prefix + ".data-00000-of-00001"
    raw = bytearray(open(data, "rb").read())
    raw[100] ^= 0xFF
    open(data, "wb").write(bytes(raw))
    with pytest.raises(Exception, match="crc32c"):
        bundle.read_bundle(prefix)


def test_crc32c_known_vectors():
    n = native()
    assert n.crc32c(b"123456789") == 0xE3069283  # standard CRC-32C check value
    assert n.crc_unmask(n.crc_mask(0x12345678)) == 0x12345678


def test_training_state_roundtrip(tmp_path):
    from tensorflow_distributed_on_gke_amd.train.optim import Adam
    cfg = model_config("tiny", src_vocab=30, tgt_vocab=30)
    m = Transformer(cfg).build("cpu", seed=1)
    opt = Adam(m.store, cfg.d_model)
    opt.m.normal_()
    opt.v.uniform_()
    opt.step.fill_(1234)
    prefix = str(tmp_path / "model_weights")
    bundle.save_weights(m.store, prefix)
    bundle.save_training_state(m.store, opt, prefix, {"epoch": 7, "batch": 3})
    m2 = Transformer(cfg).build("cpu", seed=5)
    opt2 = Adam(m2.store, cfg.d_model)
    bundle.load_weights(m2.store, prefix)
    extra = bundle.load_training_state(m2.store, opt2, prefix)
    # padding elements between params are not part of any variable
    for p in m.store.params:
        sl = slice(p.offset, p.offset + p.numel)
        assert torch.equal(opt.m[sl], opt2.m[sl]) and torch.equal(opt.v[sl], opt2.v[sl])
    assert opt2.iterations == 1234 and extra == {"epoch": 7, "batch": 3}


def test_unique_name_semantics():
    taken = {"snap", "snap_2"}
    assert unique_name("snap", taken.__contains__) == "snap_3"
    assert unique_name("x", taken.__contains__) == "x"
    assert unique_name("x", lambda s: False, number_first_name=True) == "x_1"
    assert unique_name("a", {"a.txt"}.__contains__, suffix=".txt") == "a_2.txt"


def test_model_uploader_local(tmp_path):
    cfg = model_config("tiny", src_vocab=30, tgt_vocab=30)
    m = Transformer(cfg).build("cpu", seed=1)
    st = LocalStorage(str(tmp_path / "bucket"))
    up = ModelUploader(st, "training-snapshots", str(tmp_path / "tmp"))
    up.take_snapshot(m)
    assert up.last_upload_folder == "training-snapshots/initial_model"
    assert (tmp_path / "bucket/training-snapshots/initial_model/variables/variables.index").exists()
    up.take_snapshot(m)
    assert up.last_upload_folder == "training-snapshots/weights_snapshot"
    up.take_snapshot(m)
    assert up.last_upload_folder == "training-snapshots/weights_snapshot_2"
    assert (tmp_path / "bucket/training-snapshots/weights_snapshot_2/model_weights.index").exists()
    # a second uploader picks a fresh root folder and a fresh local dir
    up2 = ModelUploader(st, "training-snapshots", str(tmp_path / "tmp"))
    up2.take_snapshot(m)
    assert up2.last_upload_folder == "training-snapshots_2/initial_model"
    assert up2.local_directory.endswith("model_uploader_2")
    m2 = Transformer(cfg).build("cpu", seed=3)
    bundle.load_weights(m2.store, str(tmp_path / "bucket/training-snapshots/weights_snapshot_2"))
    assert torch.equal(m.store.flat, m2.store.flat)
