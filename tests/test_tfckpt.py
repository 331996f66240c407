"""TF tensor-bundle checkpoints (tfckpt.py): the reference's save_weights / load_weights
format (training.py:167-170, utils.py:26-28), read and written without TensorFlow.

Parity with checkpoints written by TensorFlow itself is unpinned (none ship with the
reference and TF is not installable); these tests pin the restated format pieces that
have published known answers (CRC32C check value, LevelDB masking) and the round trip."""
import os

import numpy as np
import pytest

from neural_network_image_compression_amd import tfckpt
from neural_network_image_compression_amd import weights as W


def test_crc32c_known_answers():
    assert tfckpt.crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    assert tfckpt.crc32c(b"\x00" * 32) == 0x8A9136AA  # RFC 3720 B.4 test vector
    assert tfckpt.crc32c(bytes(range(32))) == 0x46DD794E
    assert tfckpt.mask_crc(0) == 0xA282EAD8


def test_entry_proto_roundtrip():
    raw = tfckpt.encode_entry(1, (5, 5, 32, 64), 1234, 204800, 0xDEADBEEF)
    e = tfckpt.parse_entry(raw)
    assert e["dtype"] == 1 and e["shape"] == [5, 5, 32, 64] and e["offset"] == 1234
    assert e["size"] == 204800 and e["crc32c"] == 0xDEADBEEF and not e["sliced"]


def test_table_many_keys_roundtrip(tmp_path):
    entries = {f"layer{i:03d}/kernel/.ATTRIBUTES/VARIABLE_VALUE": bytes([i % 256]) * (i % 7) for i in range(100)}
    entries[""] = b"\x08\x01"
    p = str(tmp_path / "t.index")
    tfckpt.write_table(p, entries)
    assert tfckpt.read_table(p) == entries
    data = bytearray(open(p, "rb").read())
    data[10] ^= 1
    open(p, "wb").write(bytes(data))
    with pytest.raises(ValueError):
        tfckpt.read_table(p)


def test_bundle_roundtrip_dtypes(tmp_path):
    rng = np.random.default_rng(0)
    t = {"a/kernel/.ATTRIBUTES/VARIABLE_VALUE": rng.standard_normal((3, 3, 4, 5)).astype(np.float32),
         "a/bias/.ATTRIBUTES/VARIABLE_VALUE": rng.standard_normal(5).astype(np.float32),
         "save_counter/.ATTRIBUTES/VARIABLE_VALUE": np.array(7, np.int64),
         "b/kernel/.OPTIMIZER_SLOT/optimizer/m/.ATTRIBUTES/VARIABLE_VALUE": np.ones((2,), np.float32)}
    prefix = str(tmp_path / "ck" / "encoderY")
    tfckpt.write_bundle(prefix, t)
    back = tfckpt.read_bundle(prefix)
    assert set(back) == set(t)
    for k in t:
        np.testing.assert_array_equal(back[k], t[k])
        assert back[k].dtype == t[k].dtype
    assert set(tfckpt.keras_layer_tensors(back)) == {"a/kernel", "a/bias"}
    # a flipped data byte fails the per-tensor CRC
    dp = prefix + ".data-00000-of-00001"
    raw = bytearray(open(dp, "rb").read())
    raw[3] ^= 0x40
    open(dp, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        tfckpt.read_bundle(prefix)


def test_codec_weights_via_tf_checkpoint(tmp_path):
    """ProClass.load(path) reads path+'Y' / path+'CbCr' TF checkpoints like Keras load_weights."""
    w = W.seeded_weights(3)
    for kind in ("encoder", "decoder"):
        prefix = str(tmp_path / "checkpoints" / kind)
        paths = W.save_tf(w, prefix, kind)
        assert os.path.exists(prefix + "Y.index") and os.path.exists(prefix + "CbCr.data-00000-of-00001")
        assert len(paths) == 4
        back = W.load(prefix, kind)
        sub = {k: v for k, v in w.items() if k.startswith(kind)}
        assert set(back) == set(sub)
        for k in sub:
            np.testing.assert_array_equal(back[k], sub[k])


def test_positional_layer_keys(tmp_path):
    """Functional / Sequential saves key layers as layer_with_weights-N (encoder.py:10-17 order)."""
    w = W.seeded_weights(4)
    order = ["conv1", "conv2", "conv3", "conv4", "conv8"]
    for name in W.PLANE_MODELS:
        t = {f"layer_with_weights-{i}/{var}" + tfckpt.VARIABLE_SUFFIX: w[f"encoder{name}/{l}/{var}"]
             for i, l in enumerate(order) for var in ("kernel", "bias")}
        tfckpt.write_bundle(str(tmp_path / ("enc" + name)), t)
    back = W.load(str(tmp_path / "enc"), "encoder")
    for k, v in back.items():
        np.testing.assert_array_equal(v, w[k])


def test_object_graph_written_and_decoded(tmp_path, weights_spread):
    """save_tf writes _CHECKPOINTABLE_OBJECT_GRAPH (the TrackableObjectGraph object-based
    restore walks): root -> layer attributes -> kernel / bias -> VARIABLE_VALUE with the
    checkpoint key of every tensor in the bundle; the numeric reader still skips it."""
    prefix = str(tmp_path / "ck" / "encoder")
    paths = W.save_tf(weights_spread, prefix, "encoder")
    assert len(paths) == 4
    for name, scope in (("Y", "base_encoder"), ("CbCr", "base_encoder_1")):
        nodes = tfckpt.read_object_graph(prefix + name)
        keys = set(tfckpt.read_bundle(prefix + name))
        assert tfckpt.OBJECT_GRAPH_KEY not in keys
        root = nodes[0]
        assert sorted(n for _, n in root["children"]) == ["conv1", "conv2", "conv3", "conv4", "conv8"]
        seen = set()
        for lid, lname in root["children"]:
            layer = nodes[lid]
            assert sorted(v for _, v in layer["children"]) == ["bias", "kernel"]
            for vid, vname in layer["children"]:
                (attr,) = nodes[vid]["attributes"]
                assert attr == ("VARIABLE_VALUE", f"{scope}/{lname}/{vname}",
                                f"{lname}/{vname}/.ATTRIBUTES/VARIABLE_VALUE")
                seen.add(attr[2])
        assert seen == keys
    # the loader reads the bundle back unchanged
    back = W.load(prefix, "encoder")
    for k, v in back.items():
        np.testing.assert_array_equal(v, weights_spread[k])
    # a corrupted string tensor fails its checksum
    dp = prefix + "Y.data-00000-of-00001"
    raw = bytearray(open(dp, "rb").read())
    raw[-3] ^= 0x10
    open(dp, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        tfckpt.read_object_graph(prefix + "Y")


def test_string_tensor_format():
    """TF's WriteStringTensor layout: varint64 lengths, masked CRC32C of the lengths (as
    uint32), then the bytes; the entry CRC extends over all three."""
    blob, crc = tfckpt._string_tensor_bytes([b"abc"])
    assert blob[0] == 3 and blob[5:] == b"abc"
    assert blob[1:5] == tfckpt.struct.pack("<I", tfckpt.mask_crc(tfckpt.crc32c(tfckpt.struct.pack("<I", 3))))
    c = tfckpt.crc32c(tfckpt.struct.pack("<I", 3))
    c = tfckpt.crc32c(blob[1:5], c)
    assert crc == tfckpt.crc32c(b"abc", c)
