"""TensorFlow V2 checkpoints (tensor bundles), read and written without TensorFlow.

The reference saves and restores every global variable through ``tf.train.Saver``
(``src/linear_model.py:151``; ``src/predict_3dpose.py:165-181`` restore, ``:328`` save): a
checkpoint ``<prefix>`` is

* ``<prefix>.index`` -- an immutable sorted string table (the LevelDB table format TF keeps in
  ``tensorflow/core/lib/io``): data blocks of prefix-compressed entries with restart points,
  an (empty) metaindex block, an index block of block handles, and a 48-byte footer ending in
  the magic number 0xdb4775248b80fb57; every block carries a 5-byte trailer (compression
  type, masked CRC-32C).  Key ``""`` holds the ``BundleHeaderProto`` {num_shards, endianness,
  version}; every other key is a variable name holding its ``BundleEntryProto`` {dtype,
  shape, shard_id, offset, size, masked CRC-32C of the bytes}.
* ``<prefix>.data-00000-of-00001`` -- the tensors' little-endian bytes at those offsets.
* ``checkpoint`` (next to it) -- the ``CheckpointState`` text proto naming the latest prefix.

Protos are decoded / encoded by hand (varint wire format; proto3 omits default values).  The
reader accepts uncompressed and Snappy-compressed index blocks and verifies every block and
tensor checksum (CRC-32C from libp3d's host ``p3d_crc32c``); partitioned variables (tensor
slices) are rejected.  Parity: the CRC-32C is pinned by its published check values; the table
and proto layouts follow TF's documented formats (no TF in this image, no reference
checkpoint to read: parity unpinned beyond that, tests/test_tf_bundle.py).
"""
from __future__ import annotations

import ctypes
import os
import struct

import numpy as np

TABLE_MAGIC = 0xDB4775248B80FB57
MASK_DELTA = 0xA282EAD8
RESTART_INTERVAL = 16
BLOCK_SIZE = 256 * 1024
# tensorflow DataType enum values
DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 9: np.int64, 10: np.bool_, 19: np.float16}
DT_OF = {np.dtype(v): k for k, v in DTYPES.items()}


# ---- CRC-32C ----------------------------------------------------------------------------
def crc32c(data, crc: int = 0) -> int:
    import _p3d
    buf = memoryview(data).cast("B")
    if len(buf) == 0:
        return crc
    arr = np.frombuffer(buf, np.uint8)
    return int(_p3d.lib().p3d_crc32c(arr.ctypes.data_as(ctypes.c_void_p), len(arr), crc))


def mask(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + MASK_DELTA) & 0xFFFFFFFF


def unmask(m: int) -> int:
    r = (m - MASK_DELTA) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# ---- varints / protos --------------------------------------------------------------------
def _varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos):
    shift = result = 0
    while True:
        if pos >= len(buf):
            raise ValueError("truncated varint")
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 63:
            raise ValueError("varint too long")


def _proto_fields(buf):
    """[(field, wire_type, value)]: varint -> int, 64-bit / 32-bit -> int, length -> bytes."""
    out, pos = [], 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError("unsupported proto wire type %d" % wt)
        out.append((f, wt, v))
    return out


def _pf_varint(f, v):
    return _varint(f << 3) + _varint(v) if v else b""


def _pf_bytes(f, b):
    return _varint((f << 3) | 2) + _varint(len(b)) + b


def _pf_fixed32(f, v):
    return _varint((f << 3) | 5) + struct.pack("<I", v)


def encode_header(num_shards=1, producer=1):
    version = _pf_varint(1, producer)
    return _pf_varint(1, num_shards) + _pf_bytes(3, version)          # endianness LITTLE = 0 omitted


def decode_header(buf):
    h = {"num_shards": 0, "endianness": 0, "producer": 0, "min_consumer": 0}
    for f, _, v in _proto_fields(buf):
        if f == 1:
            h["num_shards"] = v
        elif f == 2:
            h["endianness"] = v
        elif f == 3:
            for g, _, u in _proto_fields(v):
                if g == 1:
                    h["producer"] = u
                elif g == 2:
                    h["min_consumer"] = u
    return h


def encode_entry(dtype_enum, shape, offset, size, crc_masked, shard_id=0):
    shp = b"".join(_pf_bytes(2, _pf_varint(1, int(d)) if d else b"") for d in shape)
    return (_pf_varint(1, dtype_enum) + _pf_bytes(2, shp) + _pf_varint(3, shard_id) + _pf_varint(4, offset) +
            _pf_varint(5, size) + _pf_fixed32(6, crc_masked))


def decode_entry(buf):
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": 0, "slices": 0}
    for f, _, v in _proto_fields(buf):
        if f == 1:
            e["dtype"] = v
        elif f == 2:
            for g, _, dim in _proto_fields(v):
                if g == 2:
                    size = 0
                    for h, _, u in _proto_fields(dim):
                        if h == 1:
                            size = u - (1 << 64) if u >= 1 << 63 else u
                    e["shape"].append(size)
                elif g == 3 and dim:
                    raise ValueError("unknown-rank tensor shape in checkpoint")
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
        elif f == 6:
            e["crc32c"] = v
        elif f == 7:
            e["slices"] += 1
    return e


# ---- Snappy (index blocks TF wrote with compression) ----------------------------------------
def snappy_decompress(buf) -> bytes:
    n, pos = _read_varint(buf, 0)
    out = bytearray()
    while pos < len(buf):
        tag = buf[pos]
        pos += 1
        kind = tag & 3
        if kind == 0:                                   # literal
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(buf[pos:pos + nb], "little")
                pos += nb
            ln += 1
            out += buf[pos:pos + ln]
            pos += ln
            continue
        if kind == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | buf[pos]
            pos += 1
        elif kind == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 2], "little")
            pos += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(buf[pos:pos + 4], "little")
            pos += 4
        if off == 0 or off > len(out):
            raise ValueError("corrupt snappy stream")
        for _ in range(ln):                             # copies may overlap their own output
            out.append(out[-off])
    if len(out) != n:
        raise ValueError("snappy length mismatch")
    return bytes(out)


# ---- table (SSTable) -----------------------------------------------------------------------
def _block_entries(block):
    """Entries of one table block (contents without trailer) -> [(key, value)]."""
    if len(block) < 4:
        raise ValueError("table block too short")
    nres = struct.unpack_from("<I", block, len(block) - 4)[0]
    limit = len(block) - 4 - 4 * nres
    if limit < 0:
        raise ValueError("corrupt table block restarts")
    out, pos, key = [], 0, b""
    while pos < limit:
        shared, pos = _read_varint(block, pos)
        non_shared, pos = _read_varint(block, pos)
        vlen, pos = _read_varint(block, pos)
        if shared > len(key):
            raise ValueError("corrupt table entry")
        key = key[:shared] + bytes(block[pos:pos + non_shared])
        pos += non_shared
        out.append((key, bytes(block[pos:pos + vlen])))
        pos += vlen
    return out


def _read_block(data, handle_off, handle_size):
    end = handle_off + handle_size
    if end + 5 > len(data):
        raise ValueError("table block past the end of the file")
    contents = data[handle_off:end]
    ctype = data[end]
    stored = struct.unpack_from("<I", data, end + 1)[0]
    if unmask(stored) != crc32c(bytes(contents) + bytes([ctype])):
        raise ValueError("table block checksum mismatch")
    if ctype == 0:
        return bytes(contents)
    if ctype == 1:
        return snappy_decompress(bytes(contents))
    raise ValueError("unsupported table block compression %d" % ctype)


def read_table(path):
    """{key: value} of a TF / LevelDB-format sorted string table."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 48 or struct.unpack_from("<Q", data, len(data) - 8)[0] != TABLE_MAGIC:
        raise ValueError("%s: not a table (bad magic)" % path)
    foot = data[len(data) - 48:len(data) - 8]
    _, p = _read_varint(foot, 0)                        # metaindex handle (unused: no filters)
    _, p = _read_varint(foot, p)
    ioff, p = _read_varint(foot, p)
    isz, p = _read_varint(foot, p)
    out = {}
    for _, handle in _block_entries(_read_block(data, ioff, isz)):
        boff, q = _read_varint(handle, 0)
        bsz, q = _read_varint(handle, q)
        for k, v in _block_entries(_read_block(data, boff, bsz)):
            out[k] = v
    return out


class _BlockBuilder:
    def __init__(self):
        self.buf, self.restarts, self.count, self.last, self.n = bytearray(), [0], 0, b"", 0

    def add(self, key, value):
        shared = 0
        if self.count < RESTART_INTERVAL:
            n = min(len(key), len(self.last))
            while shared < n and key[shared] == self.last[shared]:
                shared += 1
        else:
            self.restarts.append(len(self.buf))
            self.count = 0
        self.buf += _varint(shared) + _varint(len(key) - shared) + _varint(len(value)) + key[shared:] + value
        self.last, self.count, self.n = key, self.count + 1, self.n + 1

    def size(self):
        return len(self.buf) + 4 * len(self.restarts) + 4

    def finish(self):
        return bytes(self.buf) + b"".join(struct.pack("<I", r) for r in self.restarts) + \
            struct.pack("<I", len(self.restarts))


def write_table(path, items):
    """Write sorted (key, value) byte pairs as an uncompressed table (TF's BundleWriter form)."""
    items = sorted(items)
    out = bytearray()

    def emit(contents):
        off = len(out)
        out.extend(contents)
        out.append(0)                                   # kNoCompression
        out.extend(struct.pack("<I", mask(crc32c(bytes(contents) + b"\x00"))))
        return _varint(off) + _varint(len(contents))

    index = _BlockBuilder()
    blk, last = _BlockBuilder(), None
    for k, v in items:
        if last is not None and k <= last:
            raise ValueError("table keys must be unique")
        blk.add(k, v)
        last = k
        if blk.size() >= BLOCK_SIZE:
            index.add(last, emit(blk.finish()))
            blk = _BlockBuilder()
    if blk.n or not items:
        index.add(last if last is not None else b"", emit(blk.finish()))
    meta = emit(_BlockBuilder().finish())
    idx = emit(index.finish())
    footer = (meta + idx).ljust(40, b"\x00") + struct.pack("<Q", TABLE_MAGIC)
    with open(path, "wb") as f:
        f.write(bytes(out) + footer)


# ---- bundles -------------------------------------------------------------------------------
def data_path(prefix, shard=0, num_shards=1):
    return "%s.data-%05d-of-%05d" % (prefix, shard, num_shards)


def write_bundle(prefix, tensors):
    """Write {name: array} as a one-shard V2 checkpoint at ``prefix``."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    items, offset = [(b"", encode_header(1))], 0
    with open(data_path(prefix), "wb") as f:
        for name in sorted(tensors, key=lambda n: n.encode()):
            a = np.asarray(tensors[name])
            dt = DT_OF.get(a.dtype.newbyteorder("="))
            if dt is None:
                raise ValueError("%s: dtype %s has no TF enum here" % (name, a.dtype))
            raw = np.ascontiguousarray(a, dtype=a.dtype.newbyteorder("<")).tobytes()
            f.write(raw)
            items.append((name.encode(), encode_entry(dt, a.shape, offset, len(raw), mask(crc32c(raw)))))
            offset += len(raw)
    write_table(prefix + ".index", items)
    return prefix


def read_bundle(prefix):
    """{name: np.ndarray} of every tensor in the V2 checkpoint at ``prefix``."""
    table = read_table(prefix + ".index")
    if b"" not in table:
        raise ValueError("%s.index: no bundle header" % prefix)
    hdr = decode_header(table[b""])
    if hdr["endianness"] != 0:
        raise ValueError("big-endian checkpoints are not supported")
    nsh = max(1, hdr["num_shards"])
    shards, out = {}, {}
    try:
        for key, val in table.items():
            if key == b"":
                continue
            e = decode_entry(val)
            name = key.decode()
            if e["slices"]:
                raise ValueError("%s: partitioned (sliced) variables are not supported" % name)
            if e["dtype"] not in DTYPES:
                raise ValueError("%s: unsupported TF dtype %d" % (name, e["dtype"]))
            sid = e["shard_id"]
            if sid not in shards:
                shards[sid] = open(data_path(prefix, sid, nsh), "rb")
            fh = shards[sid]
            fh.seek(e["offset"])
            raw = fh.read(e["size"])
            if len(raw) != e["size"]:
                raise ValueError("%s: truncated data file" % name)
            if unmask(e["crc32c"]) != crc32c(raw):
                raise ValueError("%s: tensor checksum mismatch" % name)
            a = np.frombuffer(raw, dtype=np.dtype(DTYPES[e["dtype"]]).newbyteorder("<"))
            out[name] = a.astype(a.dtype.newbyteorder("=")).reshape(e["shape"])
    finally:
        for fh in shards.values():
            fh.close()
    return out


def write_checkpoint_state(directory, latest, all_paths):
    """The ``checkpoint`` file (CheckpointState text proto) tf.train.Saver keeps."""
    lines = ['model_checkpoint_path: "%s"' % latest] + ['all_model_checkpoint_paths: "%s"' % p for p in all_paths]
    with open(os.path.join(directory or ".", "checkpoint"), "w") as f:
        f.write("\n".join(lines) + "\n")


def read_checkpoint_state(directory, latest_filename="checkpoint"):
    """model_checkpoint_path of ``directory/checkpoint`` (tf.train.get_checkpoint_state), or None."""
    p = os.path.join(directory, latest_filename)
    if not os.path.isfile(p):
        return None
    with open(p) as f:
        for line in f:
            line = line.strip()
            if line.startswith("model_checkpoint_path:"):
                v = line.split(":", 1)[1].strip().strip('"')
                return v if os.path.isabs(v) else os.path.join(directory, v)
    return None
