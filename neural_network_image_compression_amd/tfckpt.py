"""TensorFlow checkpoint (tensor bundle) reader and writer, without TensorFlow.

The reference saves each plane model with Keras ``Model.save_weights(prefix)``
(tf2_0/src/training.py:167-170) and loads it with ``load_weights`` (utils.py:26-28); with
no ``.h5`` suffix that is TF's object-based checkpoint: ``<prefix>.index`` (a LevelDB-format
table mapping tensor keys to ``BundleEntryProto`` records) and
``<prefix>.data-00000-of-00001`` (the raw little-endian tensor bytes).  Keys of a subclassed
``tf.keras.Model``'s attribute layers read ``conv1/kernel/.ATTRIBUTES/VARIABLE_VALUE``.

TensorFlow is not installable here, so this module restates the published formats
(``tensorflow/core/protobuf/tensor_bundle.proto``, ``core/lib/io/table_builder.cc`` /
``format.cc``: blocks of prefix-compressed entries + restart array + 5-byte trailer,
an index block of block handles, a 48-byte footer with magic 0xdb4775248b80fb57; masked
CRC32C).  Parity against checkpoints written by TF itself is **unpinned**: none ship
with the reference; the tests round-trip through :func:`write_bundle`.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterable, List, Tuple

import numpy as np

TABLE_MAGIC = 0xDB4775248B80FB57
FOOTER_LEN = 48
BLOCK_TRAILER = 5

#: DataType enum values (tensorflow/core/framework/types.proto) -> NumPy dtypes
DTYPES = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8, 9: np.int64,
          10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
DTYPE_IDS = {np.dtype(v): k for k, v in DTYPES.items()}

VARIABLE_SUFFIX = "/.ATTRIBUTES/VARIABLE_VALUE"


# --- CRC32C (Castagnoli), masked as LevelDB / TF do ------------------------------------
def _crc_table() -> List[int]:
    tab = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
        tab.append(c)
    return tab


_CRC_TAB = _crc_table()


def crc32c(data: bytes, crc: int = 0) -> int:
    c = crc ^ 0xFFFFFFFF
    tab = _CRC_TAB
    for b in data:
        c = tab[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def mask_crc(c: int) -> int:
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


# --- varints and protobuf wire format --------------------------------------------------
def _varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7


def _enc_varint(v: int) -> bytes:
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _proto_fields(buf: bytes) -> Iterable[Tuple[int, int, object]]:
    """(field number, wire type, value) of a serialized message; value is an int or bytes."""
    pos = 0
    while pos < len(buf):
        tag, pos = _varint(buf, pos)
        f, wt = tag >> 3, tag & 7
        if wt == 0:
            v, pos = _varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield f, wt, v


def parse_entry(buf: bytes) -> dict:
    """BundleEntryProto: dtype=1, shape=2 (TensorShapeProto: dim=2 {size=1}), shard_id=3,
    offset=4, size=5, crc32c=6 (fixed32), slices=7."""
    e = {"dtype": 0, "shape": [], "shard_id": 0, "offset": 0, "size": 0, "crc32c": None, "sliced": False}
    for f, _, v in _proto_fields(buf):
        if f == 1:
            e["dtype"] = v
        elif f == 2:
            for f2, _, d in _proto_fields(v):
                if f2 == 2:
                    size = 0
                    for f3, _, s in _proto_fields(d):
                        if f3 == 1:
                            size = s - (1 << 64) if s >= 1 << 63 else s
                    e["shape"].append(size)
        elif f == 3:
            e["shard_id"] = v
        elif f == 4:
            e["offset"] = v
        elif f == 5:
            e["size"] = v
        elif f == 6:
            e["crc32c"] = v
        elif f == 7:
            e["sliced"] = True
    return e


def _enc_field(f: int, wt: int, payload: bytes) -> bytes:
    return _enc_varint(f << 3 | wt) + payload


def encode_entry(dtype: int, shape: Tuple[int, ...], offset: int, size: int, crc: int) -> bytes:
    dims = b"".join(_enc_field(2, 2, _enc_varint(len(d)) + d)
                    for d in (_enc_field(1, 0, _enc_varint(s)) for s in shape))
    out = _enc_field(1, 0, _enc_varint(dtype))
    out += _enc_field(2, 2, _enc_varint(len(dims)) + dims)
    if offset:
        out += _enc_field(4, 0, _enc_varint(offset))
    out += _enc_field(5, 0, _enc_varint(size))
    out += _enc_field(6, 5, struct.pack("<I", crc))
    return out


# --- LevelDB table format ---------------------------------------------------------------
def _read_block(data: bytes, offset: int, size: int, verify: bool) -> bytes:
    block = data[offset:offset + size]
    ctype = data[offset + size]
    if ctype != 0:
        raise ValueError(f"compressed table block (type {ctype}) is not supported")
    if verify:
        stored = struct.unpack_from("<I", data, offset + size + 1)[0]
        if mask_crc(crc32c(data[offset:offset + size + 1])) != stored:
            raise ValueError(f"table block at {offset}: CRC mismatch")
    return block


def _block_entries(block: bytes) -> Iterable[Tuple[bytes, bytes]]:
    nrestart = struct.unpack_from("<I", block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrestart
    pos, key = 0, b""
    while pos < end:
        shared, pos = _varint(block, pos)
        non_shared, pos = _varint(block, pos)
        vlen, pos = _varint(block, pos)
        key = key[:shared] + block[pos:pos + non_shared]
        pos += non_shared
        yield key, block[pos:pos + vlen]
        pos += vlen


def read_table(path: str, verify: bool = True) -> Dict[str, bytes]:
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < FOOTER_LEN:
        raise ValueError(f"{path}: too short for a table")
    footer = data[-FOOTER_LEN:]
    if struct.unpack_from("<Q", footer, FOOTER_LEN - 8)[0] != TABLE_MAGIC:
        raise ValueError(f"{path}: bad table magic")
    pos = 0
    _, pos = _varint(footer, pos)  # metaindex handle (unused)
    _, pos = _varint(footer, pos)
    idx_off, pos = _varint(footer, pos)
    idx_size, pos = _varint(footer, pos)
    out: Dict[str, bytes] = {}
    for _, handle in _block_entries(_read_block(data, idx_off, idx_size, verify)):
        off, p = _varint(handle, 0)
        size, _ = _varint(handle, p)
        for k, v in _block_entries(_read_block(data, off, size, verify)):
            out[k.decode()] = v
    return out


def _build_block(items: List[Tuple[bytes, bytes]], restart_interval: int = 16) -> bytes:
    out, restarts, prev = bytearray(), [], b""
    for i, (k, v) in enumerate(items):
        if i % restart_interval == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(prev)) and k[shared] == prev[shared]:
                shared += 1
        out += _enc_varint(shared) + _enc_varint(len(k) - shared) + _enc_varint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts.append(0)
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def write_table(path: str, entries: Dict[str, bytes]) -> None:
    """One data block, an empty metaindex block, an index block, the footer (no compression)."""
    buf = bytearray()

    def put(block: bytes) -> bytes:
        off = len(buf)
        buf.extend(block)
        trailer = b"\x00"
        buf.extend(trailer + struct.pack("<I", mask_crc(crc32c(block + trailer))))
        return _enc_varint(off) + _enc_varint(len(block))

    items = sorted((k.encode(), v) for k, v in entries.items())
    data_h = put(_build_block(items))
    meta_h = put(_build_block([]))
    last = items[-1][0] if items else b""
    index_h = put(_build_block([(last, data_h)]))
    footer = meta_h + index_h
    footer += b"\x00" * (FOOTER_LEN - 8 - len(footer)) + struct.pack("<Q", TABLE_MAGIC)
    buf.extend(footer)
    with open(path, "wb") as f:
        f.write(bytes(buf))


# --- tensor bundles -------------------------------------------------------------------
def read_bundle(prefix: str, verify: bool = True) -> Dict[str, np.ndarray]:
    """Every tensor of ``<prefix>.index`` / ``<prefix>.data-*``: {key: array}.  The header
    entry (empty key) and non-numeric entries (the object graph is a DT_STRING) are skipped."""
    table = read_table(prefix + ".index", verify)
    header = table.pop("", b"")
    num_shards = 1
    for f, _, v in _proto_fields(header):
        if f == 1:
            num_shards = v
        elif f == 2 and v != 0:
            raise ValueError(f"{prefix}: big-endian bundles are not supported")
    shards: Dict[int, bytes] = {}
    out: Dict[str, np.ndarray] = {}
    for key, raw in table.items():
        e = parse_entry(raw)
        if e["sliced"]:
            raise ValueError(f"{prefix}: partitioned variable {key!r} is not supported")
        if e["dtype"] not in DTYPES:
            continue
        sid = e["shard_id"]
        if sid not in shards:
            with open(f"{prefix}.data-{sid:05d}-of-{num_shards:05d}", "rb") as f:
                shards[sid] = f.read()
        blob = shards[sid][e["offset"]:e["offset"] + e["size"]]
        if len(blob) != e["size"]:
            raise ValueError(f"{prefix}: tensor {key!r} runs past the end of its data shard")
        if verify and e["crc32c"] is not None and mask_crc(crc32c(blob)) != e["crc32c"]:
            raise ValueError(f"{prefix}: tensor {key!r} fails its CRC32C")
        out[key] = np.frombuffer(blob, dtype=np.dtype(DTYPES[e["dtype"]]).newbyteorder("<")).reshape(e["shape"]).copy()
    return out


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray]) -> List[str]:
    """Single-shard little-endian bundle of ``tensors`` (keys written in sorted order)."""
    d = os.path.dirname(prefix)
    if d:
        os.makedirs(d, exist_ok=True)
    data = bytearray()
    entries: Dict[str, bytes] = {"": _enc_field(1, 0, _enc_varint(1)) + _enc_field(3, 2, _enc_varint(2) +
                                                                                    _enc_field(1, 0, _enc_varint(1)))}
    for key in sorted(tensors):
        a = np.ascontiguousarray(tensors[key])
        if a.dtype not in DTYPE_IDS:
            raise TypeError(f"write_bundle: dtype {a.dtype} of {key!r} not supported")
        blob = a.astype(a.dtype.newbyteorder("<"), copy=False).tobytes()
        entries[key] = encode_entry(DTYPE_IDS[a.dtype], a.shape, len(data), len(blob), mask_crc(crc32c(blob)))
        data.extend(blob)
    write_table(prefix + ".index", entries)
    dpath = prefix + ".data-00000-of-00001"
    with open(dpath, "wb") as f:
        f.write(bytes(data))
    return [prefix + ".index", dpath]


def keras_layer_tensors(bundle: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
    """Object-based Keras keys ``<layer>/<kernel|bias>/.ATTRIBUTES/VARIABLE_VALUE`` ->
    ``<layer>/<kernel|bias>``; optimizer slots, the save counter and the object graph drop out."""
    out = {}
    for key, v in bundle.items():
        if key.endswith(VARIABLE_SUFFIX) and "/.OPTIMIZER_SLOT/" not in key:
            name = key[:-len(VARIABLE_SUFFIX)]
            if name.count("/") == 1:
                out[name] = v
    return out
