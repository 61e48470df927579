"""TFRecord IO (libkge_hip.so kge_tfrecord_*) checked against Google's protobuf runtime building the
tf.train.Example messages from the published example.proto/feature.proto schema, and against the
CRC-32C check value of RFC 3720 (0xE3069283 for "123456789"). TensorFlow itself is absent here, so
the framing is pinned by those two independent sources."""
import os
import struct

import numpy as np
import pytest

from customknowledgegraphembedding_amd import _lib
from customknowledgegraphembedding_amd.tfrecord import (TFRecordDataset, TFRecordWriter, load_batches,
                                                         reshape_function, write_file_tfrecords)


def _example_classes():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fd = descriptor_pb2.FileDescriptorProto(name="kge_test_example.proto", package="tensorflow", syntax="proto3")
    F = descriptor_pb2.FieldDescriptorProto
    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m
    R, O = F.LABEL_REPEATED, F.LABEL_OPTIONAL
    msg("BytesList", [("value", 1, F.TYPE_BYTES, R, None)])
    msg("FloatList", [("value", 1, F.TYPE_FLOAT, R, None)])
    msg("Int64List", [("value", 1, F.TYPE_INT64, R, None)])
    feat = msg("Feature", [("bytes_list", 1, F.TYPE_MESSAGE, O, ".tensorflow.BytesList"),
                           ("float_list", 2, F.TYPE_MESSAGE, O, ".tensorflow.FloatList"),
                           ("int64_list", 3, F.TYPE_MESSAGE, O, ".tensorflow.Int64List")])
    feat.oneof_decl.add(name="kind")
    for f in feat.field:
        f.oneof_index = 0
    fs = fd.message_type.add(name="Features")
    entry = fs.nested_type.add(name="FeatureEntry")
    entry.options.map_entry = True
    entry.field.add(name="key", number=1, type=F.TYPE_STRING, label=O)
    entry.field.add(name="value", number=2, type=F.TYPE_MESSAGE, label=O, type_name=".tensorflow.Feature")
    fs.field.add(name="feature", number=1, type=F.TYPE_MESSAGE, label=R, type_name=".tensorflow.Features.FeatureEntry")
    msg("Example", [("features", 1, F.TYPE_MESSAGE, O, ".tensorflow.Features")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("tensorflow.Example"))


Example = _example_classes()


def _crc(b):
    return _lib.load().kge_crc32c(b, len(b))


def _masked(b):
    c = _crc(b)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _frame(data):
    hdr = struct.pack("<Q", len(data))
    return hdr + struct.pack("<I", _masked(hdr)) + data + struct.pack("<I", _masked(data))


def _make_example(pos, neg, w, mode):
    ex = Example()
    f = ex.features.feature
    f["positive_sample"].int64_list.value.extend(int(v) for v in pos)
    f["negative_sample"].int64_list.value.extend(int(v) for v in neg)
    f["subsampling_weight"].float_list.value.extend(float(v) for v in w)
    f["mode"].int64_list.value.extend(int(v) for v in mode)
    return ex


def _batch(seed, B=8, N=16, E=40943):
    g = np.random.RandomState(seed)
    pos = g.randint(E, size=(B, 3)).astype(np.int64)
    neg = g.randint(E, size=(B, N)).astype(np.int64)
    w = g.rand(B, 1).astype(np.float32)
    mode = np.full(B, seed % 2, dtype=np.int64)
    return pos, neg, w, mode


def test_crc32c_check_value():
    assert _crc(b"123456789") == 0xE3069283
    assert _crc(b"") == 0
    big = bytes(range(256)) * 37
    # slicing-by-8 path vs bytewise path on the same data split at odd offsets
    assert _crc(big) == _crc(big[:3] + big[3:])


def test_writer_bytes_match_protobuf_deterministic(tmp_path):
    pos, neg, w, mode = _batch(0)
    path = str(tmp_path / "a.tfrec")
    with TFRecordWriter(path) as wr:
        wr.write(np.hstack(pos), np.hstack(neg), np.hstack(w), mode)
    data = open(path, "rb").read()
    want = _make_example(pos.reshape(-1), neg.reshape(-1), w.reshape(-1), mode).SerializeToString(deterministic=True)
    assert data == _frame(want)


def test_reader_parses_protobuf_examples_any_order(tmp_path):
    path = str(tmp_path / "b.tfrec")
    batches = [_batch(s) for s in range(3)]
    with open(path, "wb") as f:
        for i, (pos, neg, w, mode) in enumerate(batches):
            ex = _make_example(pos.reshape(-1), neg.reshape(-1), w.reshape(-1), mode)
            f.write(_frame(ex.SerializeToString(deterministic=bool(i % 2))))
    got = list(TFRecordDataset(path))
    assert len(got) == 3
    for ex, (pos, neg, w, mode) in zip(got, batches):
        p, n, ww, m = reshape_function(ex, 8)
        assert np.array_equal(p.numpy(), pos) and np.array_equal(n.numpy(), neg)
        assert np.array_equal(ww.numpy(), w) and np.array_equal(m.numpy(), mode)


def test_reader_unpacked_and_negative_values(tmp_path):
    # hand-encoded Int64List with unpacked (wire type 0) values, incl. a negative (10-byte varint)
    def varint(v):
        v &= (1 << 64) - 1
        out = bytearray()
        while v >= 0x80:
            out.append((v & 0x7F) | 0x80)
            v >>= 7
        out.append(v)
        return bytes(out)

    def ld(field, body):
        return varint(field << 3 | 2) + varint(len(body)) + body

    vals = [5, -1, 1 << 40]
    i64 = b"".join(varint(1 << 3 | 0) + varint(v) for v in vals)
    feat = ld(3, i64)
    entry = ld(1, b"mode") + ld(2, feat)
    unknown = varint(7 << 3 | 0) + varint(99)  # unknown field inside Features: skipped
    ex = ld(1, ld(1, entry) + unknown)
    path = str(tmp_path / "c.tfrec")
    open(path, "wb").write(_frame(ex))
    (got,) = list(TFRecordDataset(path))
    assert got["mode"].tolist() == vals
    assert got["positive_sample"].size == 0


def test_crc_mismatch_and_truncation_raise(tmp_path):
    pos, neg, w, mode = _batch(1)
    path = str(tmp_path / "d.tfrec")
    with TFRecordWriter(path) as wr:
        wr.write(pos, neg, w, mode)
    raw = bytearray(open(path, "rb").read())
    raw[20] ^= 1
    bad = str(tmp_path / "bad.tfrec")
    open(bad, "wb").write(bytes(raw))
    with pytest.raises(_lib.KGEHipError, match="CRC"):
        list(TFRecordDataset(bad))
    assert len(list(TFRecordDataset(bad, verify_crc=False))) == 1
    cut = str(tmp_path / "cut.tfrec")
    open(cut, "wb").write(bytes(raw[:-7]))
    with pytest.raises(_lib.KGEHipError, match="truncated"):
        list(TFRecordDataset(cut, verify_crc=False))


def test_wrong_list_type_raises(tmp_path):
    ex = Example()
    ex.features.feature["mode"].float_list.value.extend([1.0])
    path = str(tmp_path / "e.tfrec")
    open(path, "wb").write(_frame(ex.SerializeToString()))
    with pytest.raises(_lib.KGEHipError, match="wrong list type"):
        list(TFRecordDataset(path))


def test_write_file_tfrecords_and_repeat(tmp_path):
    batches = [_batch(s) for s in range(7)] + [_batch(9, B=5)]
    out = tmp_path / "wn18rr"
    out.mkdir()
    paths = write_file_tfrecords(batches, str(out), batch_size=8, split_number=3)
    assert [os.path.basename(p) for p in paths] == ["wn18rr-0.tfrec", "wn18rr-1.tfrec", "wn18rr-2.tfrec"]
    it = load_batches(paths, 8, repeat=True, prefetch=2)
    seen = [next(it) for _ in range(8)]  # 6 written (8 // 3 = 2 per file) then repeat
    for k in range(8):
        pos, neg, w, mode = batches[k % 6]
        assert np.array_equal(seen[k][1].numpy(), neg)
        assert np.array_equal(seen[k][2].numpy(), w)
    it.close()
    assert len(list(load_batches(paths, 8, repeat=False, prefetch=0))) == 6


def test_reshape_rejects_bad_batch():
    with pytest.raises(ValueError):
        reshape_function({"positive_sample": np.zeros(9, np.int64), "negative_sample": np.zeros(8, np.int64),
                          "subsampling_weight": np.zeros(4, np.float32), "mode": np.zeros(4, np.int64)}, 4)
