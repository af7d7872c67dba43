"""Ray Data TFRecords (modelled on python/ray/data/tests/test_tfrecords.py): round trip,
wire-format parity against the protobuf library's own encoder/decoder (Example messages
built from a runtime descriptor, since TensorFlow is not installed), CRC checking, gzip."""

import gzip
import os

import numpy as np
import pytest

import ray_amd as ray
from ray_amd import data as rd


@pytest.fixture(scope="module", autouse=True)
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _example_classes():
    """tf.train.Example / Features / Feature as dynamic protobuf messages (same field
    numbers and packing as tensorflow/core/example/{example,feature}.proto)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fdp = descriptor_pb2.FileDescriptorProto(name="ex_test.proto", package="tfx",
                                             syntax="proto3")
    F = descriptor_pb2.FieldDescriptorProto

    def msg(name, fields, nested=()):
        m = fdp.message_type.add(name=name)
        for fname, num, typ, label, tname, oneof in fields:
            f = m.field.add(name=fname, number=num, type=typ, label=label)
            if tname:
                f.type_name = tname
            if oneof is not None:
                f.oneof_index = oneof
        return m

    rep, opt = F.LABEL_REPEATED, F.LABEL_OPTIONAL
    msg("BytesList", [("value", 1, F.TYPE_BYTES, rep, None, None)])
    msg("FloatList", [("value", 1, F.TYPE_FLOAT, rep, None, None)])
    msg("Int64List", [("value", 1, F.TYPE_INT64, rep, None, None)])
    feat = msg("Feature", [("bytes_list", 1, F.TYPE_MESSAGE, opt, ".tfx.BytesList", 0),
                           ("float_list", 2, F.TYPE_MESSAGE, opt, ".tfx.FloatList", 0),
                           ("int64_list", 3, F.TYPE_MESSAGE, opt, ".tfx.Int64List", 0)])
    feat.oneof_decl.add(name="kind")
    feats = msg("Features", [("feature", 1, F.TYPE_MESSAGE, rep, ".tfx.Features.FeatureEntry",
                              None)])
    entry = feats.nested_type.add(name="FeatureEntry")
    entry.field.add(name="key", number=1, type=F.TYPE_STRING, label=opt)
    entry.field.add(name="value", number=2, type=F.TYPE_MESSAGE, label=opt,
                    type_name=".tfx.Feature")
    entry.options.map_entry = True
    msg("Example", [("features", 1, F.TYPE_MESSAGE, opt, ".tfx.Features", None)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("tfx.Example"))


def test_round_trip(tmp_path):
    rows = [{"i": 3, "f": 1.5, "b": b"\x00ab", "s": "héllo", "il": [1, -2, 3],
             "fl": [0.25, -1.0]},
            {"i": -7, "f": 2.0, "b": b"", "s": "x", "il": [2 ** 40], "fl": [3.5, 4.5, 5.5]}]
    rd.from_items(rows).write_tfrecords(str(tmp_path))
    files = sorted(os.listdir(tmp_path))
    assert files and all(f.endswith(".tfrecords") for f in files)
    out = sorted(rd.read_tfrecords(str(tmp_path)).take_all(), key=lambda r: r["f"])
    assert [r["i"] for r in out] == [3, -7]
    assert [r["b"] for r in out] == [b"\x00ab", b""]
    assert [r["s"] for r in out] == ["héllo".encode(), b"x"]
    # a one-value list reads back as a scalar (reference: _get_feature_value unwraps
    # single values)
    assert list(out[0]["il"]) == [1, -2, 3] and np.atleast_1d(out[1]["il"]).tolist() == \
        [2 ** 40]
    np.testing.assert_allclose(out[1]["fl"], [3.5, 4.5, 5.5])


def test_wire_format_parity_with_protobuf(tmp_path):
    from ray_amd._native import _core
    from ray_amd.data.tfrecords import decode_example, encode_example

    Example = _example_classes()
    ex = Example()
    ex.features.feature["ints"].int64_list.value.extend([5, -1, 300])
    ex.features.feature["floats"].float_list.value.extend([0.5, 2.25])
    ex.features.feature["blob"].bytes_list.value.append(b"payload")
    ex.features.feature["empty"].bytes_list.SetInParent()
    blob = ex.SerializeToString()
    got = decode_example(blob)
    assert got["ints"] == (3, [5, -1, 300])
    assert got["floats"] == (2, [0.5, 2.25])
    assert got["blob"] == (1, [b"payload"])
    assert got["empty"] == (1, [])
    # our encoder's bytes parse with protobuf to the same values
    back = Example.FromString(encode_example({"ints": [5, -1, 300], "floats": [0.5, 2.25],
                                              "blob": b"payload"}))
    assert list(back.features.feature["ints"].int64_list.value) == [5, -1, 300]
    assert list(back.features.feature["floats"].float_list.value) == [0.5, 2.25]
    assert list(back.features.feature["blob"].bytes_list.value) == [b"payload"]
    # a file of protobuf-serialized Examples reads through Ray Data
    exs = []
    for k in range(5):
        e = Example()
        e.features.feature["k"].int64_list.value.append(k)
        e.features.feature["v"].float_list.value.extend([k, k + 0.5])
        exs.append(e.SerializeToString())
    (tmp_path / "pb.tfrecords").write_bytes(_core.tfrecord_encode(exs))
    rows = rd.read_tfrecords(str(tmp_path / "pb.tfrecords")).take_all()
    assert [r["k"] for r in rows] == list(range(5))
    np.testing.assert_allclose(rows[4]["v"], [4.0, 4.5])


def test_crc_verification_and_gzip(tmp_path):
    from ray_amd._native import _core

    assert _core.crc32c(b"123456789") == 0xE3069283  # CRC-32C check value
    rd.from_items([{"x": i} for i in range(10)]).repartition(1).write_tfrecords(
        str(tmp_path / "plain"))
    (f,) = os.listdir(tmp_path / "plain")
    raw = bytearray((tmp_path / "plain" / f).read_bytes())
    n0 = int.from_bytes(raw[:8], "little")
    raw[12 + n0] ^= 0xFF  # corrupt the first record's payload CRC
    (tmp_path / "bad.tfrecords").write_bytes(bytes(raw))
    with pytest.raises(Exception, match="CRC"):
        rd.read_tfrecords(str(tmp_path / "bad.tfrecords")).take_all()
    assert len(rd.read_tfrecords(str(tmp_path / "bad.tfrecords"),
                                 verify=False).take_all()) == 10
    rd.from_items([{"x": i} for i in range(10)]).write_tfrecords(
        str(tmp_path / "gz"), compression="gzip")
    names = os.listdir(tmp_path / "gz")
    assert all(n.endswith(".tfrecords.gz") for n in names)
    gzip.decompress((tmp_path / "gz" / names[0]).read_bytes())  # a real gzip stream
    xs = sorted(r["x"] for r in rd.read_tfrecords(str(tmp_path / "gz")).take_all())
    assert xs == list(range(10))
