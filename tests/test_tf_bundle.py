"""TensorFlow V2 checkpoint (tensor bundle) I/O without TensorFlow (3d-pose-baseline_amd/tf_bundle.py).

The reference saves / restores through tf.train.Saver (src/linear_model.py:151,
src/predict_3dpose.py:165-181,328).  TF is not in this image and the reference ships no
checkpoint, so the format pieces are pinned where published values exist -- CRC-32C check
values (RFC 3720 B.4 and the usual "123456789" check), a hand-assembled Snappy stream, a
table and a BundleEntryProto assembled byte by byte from the format spec -- and the rest by
round trips (parity unpinned against TF itself).  CPU only: p3d_crc32c is host code."""
import os
import struct
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "3d-pose-baseline_amd"))

tb = pytest.importorskip("tf_bundle")


def test_crc32c_check_values():
    assert tb.crc32c(b"123456789") == 0xE3069283
    assert tb.crc32c(bytes(32)) == 0x8A9136AA                       # RFC 3720 B.4
    assert tb.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert tb.crc32c(bytes(range(32))) == 0x46DD794E
    assert tb.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    data = np.random.default_rng(0).integers(0, 256, 100003, dtype=np.uint8).tobytes()
    assert tb.crc32c(data[37:], tb.crc32c(data[:37])) == tb.crc32c(data)   # continuation
    assert tb.unmask(tb.mask(0x12345678)) == 0x12345678


def test_snappy_hand_stream():
    # "abcabcabcabc": length 12, literal "abc", copy (1-byte offset) of 9 bytes from offset 3
    stream = bytes([12, (3 - 1) << 2]) + b"abc" + bytes([((9 - 4) << 2) | 1, 3])
    assert tb.snappy_decompress(stream) == b"abcabcabcabc"
    # a long literal (length in one extra byte), a 2-byte-offset copy of 64, a 1-byte one of 6
    lit = bytes(range(70))
    stream = bytes([0x8C, 0x01]) + bytes([60 << 2, 69]) + lit + bytes([(63 << 2) | 2, 70, 0, ((6 - 4) << 2) | 1, 70])
    assert tb.snappy_decompress(stream) == lit + lit


def _block(entries, restarts):
    body = b""
    for shared, key, value in entries:
        body += bytes([shared, len(key) - shared, len(value)]) + key[shared:] + value
    return body + b"".join(struct.pack("<I", r) for r in restarts) + struct.pack("<I", len(restarts))


def _trailer(contents):
    return b"\x00" + struct.pack("<I", tb.mask(tb.crc32c(contents + b"\x00")))


def test_read_hand_assembled_table():
    # one data block: "" -> "h", "ab" -> "1", "ac" -> "22" (prefix-shared), restarts [0]
    data = _block([(0, b"", b"h"), (0, b"ab", b"1"), (1, b"ac", b"22")], [0])
    meta = _block([], [0])
    f = data + _trailer(data)
    moff = len(f)
    f += meta + _trailer(meta)
    ioff = len(f)
    index = _block([(0, b"ac", bytes([0, len(data)]))], [0])        # handle: varint offset, size
    f += index + _trailer(index)
    footer = bytes([moff, len(meta), ioff, len(index)]).ljust(40, b"\x00") + struct.pack("<Q", tb.TABLE_MAGIC)
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "p3d_hand.index")
    with open(path, "wb") as fh:
        fh.write(f + footer)
    assert tb.read_table(path) == {b"": b"h", b"ab": b"1", b"ac": b"22"}
    with open(path, "r+b") as fh:                                     # flip a byte of the data block
        fh.seek(3)
        fh.write(b"\x7f")
    with pytest.raises(ValueError, match="checksum"):
        tb.read_table(path)


def test_decode_hand_encoded_entry():
    shape = bytes([0x12, 2, 0x08, 2, 0x12, 2, 0x08, 3])               # dim {size: 2} dim {size: 3}
    buf = bytes([0x08, 1, 0x12, len(shape)]) + shape + bytes([0x20, 4, 0x28, 24, 0x35]) + struct.pack("<I", 0xDEADBEEF)
    e = tb.decode_entry(buf)
    assert (e["dtype"], e["shape"], e["shard_id"], e["offset"], e["size"], e["crc32c"]) == (1, [2, 3], 0, 4, 24, 0xDEADBEEF)
    assert tb.decode_entry(tb.encode_entry(1, (2, 3), 4, 24, 0xDEADBEEF)) == e
    h = tb.decode_header(tb.encode_header(1))
    assert h["num_shards"] == 1 and h["endianness"] == 0 and h["producer"] == 1


@pytest.mark.parametrize("nblock", [1, 3])
def test_bundle_round_trip(tmp_path, nblock, monkeypatch):
    if nblock > 1:
        monkeypatch.setattr(tb, "BLOCK_SIZE", 64)                     # force several data blocks
    rng = np.random.default_rng(1)
    state = {"linear_model/w1": rng.standard_normal((32, 1024)).astype(np.float32),
             "linear_model/w1/Adam": rng.standard_normal((32, 1024)).astype(np.float32),
             "linear_model/w1/Adam_1": rng.random((32, 1024)).astype(np.float32),
             "linear_model/b1": rng.standard_normal(1024).astype(np.float32),
             "global_step": np.array(4874200, np.int32), "beta1_power": np.array(0.9 ** 7, np.float32),
             "learning_rate": np.array(1e-3, np.float32), "x64": np.arange(5, dtype=np.int64),
             "f64": rng.standard_normal((3, 0, 2))}
    for i in range(40):
        state["extra/v%02d" % i] = np.full((i % 3 + 1,), i, np.float32)
    prefix = str(tmp_path / "checkpoint-7")
    tb.write_bundle(prefix, state)
    assert os.path.isfile(prefix + ".index") and os.path.isfile(prefix + ".data-00000-of-00001")
    got = tb.read_bundle(prefix)
    assert set(got) == set(state)
    for k, v in state.items():
        assert got[k].dtype == v.dtype and got[k].shape == v.shape, k
        np.testing.assert_array_equal(got[k], v)
    raw = bytearray(open(prefix + ".data-00000-of-00001", "rb").read())
    raw[100] ^= 1
    open(prefix + ".data-00000-of-00001", "wb").write(bytes(raw))
    with pytest.raises(ValueError, match="checksum"):
        tb.read_bundle(prefix)
    tb.write_checkpoint_state(str(tmp_path), "checkpoint-7", ["checkpoint-5", "checkpoint-7"])
    assert tb.read_checkpoint_state(str(tmp_path)) == prefix
