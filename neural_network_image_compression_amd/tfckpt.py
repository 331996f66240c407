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
CRC32C).  Bundles written here also carry the ``_CHECKPOINTABLE_OBJECT_GRAPH`` entry
(a scalar DT_STRING holding a serialized ``TrackableObjectGraph``,
``tensorflow/core/protobuf/trackable_object_graph.proto``) that TF2's object-based restore
(``Model.load_weights``, utils.py:26-28) walks to match checkpoint keys to variables:
root -> one child per layer attribute -> ``kernel`` / ``bias`` -> a ``VARIABLE_VALUE``
attribute with its checkpoint key.  Parity against checkpoints written, or read, by TF
itself is **unpinned**: none ship with the reference and TF is absent; the tests
round-trip through :func:`write_bundle` and decode the object graph back.
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
OBJECT_GRAPH_KEY = "_CHECKPOINTABLE_OBJECT_GRAPH"
DT_STRING = 7


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


def _enc_bytes(f: int, b: bytes) -> bytes:
    return _enc_field(f, 2, _enc_varint(len(b)) + b)


def encode_object_graph(variable_keys: Iterable[str], scope: str = "") -> bytes:
    """TrackableObjectGraph of a subclassed Keras model whose attribute layers own the
    variables ``<layer>/<var>`` (keys ``<layer>/<var>/.ATTRIBUTES/VARIABLE_VALUE``):
    nodes = [root, layer..., variable...]; TrackableObject: children = 1 (ObjectReference:
    node_id = 1, local_name = 2), attributes = 2 (SerializedTensor: name = 1, full_name = 2,
    checkpoint_key = 3).  ``scope`` prefixes the informational full names."""
    names = sorted(k[:-len(VARIABLE_SUFFIX)] if k.endswith(VARIABLE_SUFFIX) else k for k in variable_keys)
    layers: Dict[str, List[str]] = {}
    for n in names:
        layer, var = n.split("/")
        layers.setdefault(layer, []).append(var)
    layer_ids = {layer: 1 + i for i, layer in enumerate(layers)}
    var_ids, nid = {}, 1 + len(layers)
    for layer, vars_ in layers.items():
        for v in vars_:
            var_ids[(layer, v)] = nid
            nid += 1

    def ref(node_id: int, local: str) -> bytes:
        return _enc_bytes(1, _enc_field(1, 0, _enc_varint(node_id)) + _enc_bytes(2, local.encode()))

    nodes = [b"".join(ref(layer_ids[layer], layer) for layer in layers)]
    for layer, vars_ in layers.items():
        nodes.append(b"".join(ref(var_ids[(layer, v)], v) for v in vars_))
    for layer, vars_ in layers.items():
        for v in vars_:
            full = "/".join(p for p in (scope, layer, v) if p)
            tensor = (_enc_bytes(1, b"VARIABLE_VALUE") + _enc_bytes(2, full.encode()) +
                      _enc_bytes(3, f"{layer}/{v}{VARIABLE_SUFFIX}".encode()))
            nodes.append(_enc_bytes(2, tensor))
    return b"".join(_enc_bytes(1, n) for n in nodes)


def decode_object_graph(buf: bytes) -> List[dict]:
    """Inverse of :func:`encode_object_graph` (any TrackableObjectGraph): per node
    {"children": [(node_id, local_name)], "attributes": [(name, full_name, checkpoint_key)]}."""
    nodes = []
    for f, _, node in _proto_fields(buf):
        if f != 1:
            continue
        children, attrs = [], []
        for f2, _, v in _proto_fields(node):
            if f2 == 1:
                d = {k: x for k, _, x in _proto_fields(v)}
                children.append((d.get(1, 0), d.get(2, b"").decode()))
            elif f2 == 2:
                d = {k: x for k, _, x in _proto_fields(v)}
                attrs.append(tuple(d.get(k, b"").decode() for k in (1, 2, 3)))
        nodes.append({"children": children, "attributes": attrs})
    return nodes


def _string_tensor_bytes(elems: List[bytes]) -> Tuple[bytes, int]:
    """TF's WriteStringTensor (tensor_bundle.cc): varint64 lengths, the masked CRC32C of the
    lengths taken as uint32s, then the bytes; returns (blob, crc32c over all of it as TF
    extends it: the uint32 lengths, the length checksum, the string bytes)."""
    lengths, crc = b"", 0
    for e in elems:
        lengths += _enc_varint(len(e))
        crc = crc32c(struct.pack("<I", len(e)), crc)
    lcrc = struct.pack("<I", mask_crc(crc))
    crc = crc32c(lcrc, crc)
    for e in elems:
        crc = crc32c(e, crc)
    return lengths + lcrc + b"".join(elems), crc


def _read_string_scalar(blob: bytes, verify: bool, key: str) -> bytes:
    n, pos = _varint(blob, 0)
    if verify:
        crc = crc32c(struct.pack("<I", n))
        if struct.unpack_from("<I", blob, pos)[0] != mask_crc(crc):
            raise ValueError(f"string tensor {key!r}: length checksum mismatch")
    return bytes(blob[pos + 4:pos + 4 + n])


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


def read_object_graph(prefix: str, verify: bool = True) -> List[dict]:
    """The decoded ``_CHECKPOINTABLE_OBJECT_GRAPH`` of a bundle (KeyError if it has none)."""
    table = read_table(prefix + ".index", verify)
    header = table.get("", b"")
    num_shards = next((v for f, _, v in _proto_fields(header) if f == 1), 1)
    e = parse_entry(table[OBJECT_GRAPH_KEY])
    if e["dtype"] != DT_STRING or e["shape"]:
        raise ValueError(f"{prefix}: {OBJECT_GRAPH_KEY} is not a scalar DT_STRING")
    with open(f"{prefix}.data-{e['shard_id']:05d}-of-{num_shards:05d}", "rb") as f:
        f.seek(e["offset"])
        blob = f.read(e["size"])
    payload = _read_string_scalar(blob, verify, OBJECT_GRAPH_KEY)
    if verify and e["crc32c"] is not None:
        # the entry CRC of a string tensor extends over the lengths as uint32s, not their varints
        rebuilt, crc = _string_tensor_bytes([payload])
        if rebuilt != blob or mask_crc(crc) != e["crc32c"]:
            raise ValueError(f"{prefix}: {OBJECT_GRAPH_KEY} fails its CRC32C")
    return decode_object_graph(payload)


def write_bundle(prefix: str, tensors: Dict[str, np.ndarray], object_graph: bytes = None) -> List[str]:
    """Single-shard little-endian bundle of ``tensors`` (keys written in sorted order), plus
    ``object_graph`` (a serialized TrackableObjectGraph) as the scalar DT_STRING entry
    ``_CHECKPOINTABLE_OBJECT_GRAPH`` when given."""
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
    if object_graph is not None:
        blob, crc = _string_tensor_bytes([object_graph])
        entries[OBJECT_GRAPH_KEY] = encode_entry(DT_STRING, (), len(data), len(blob), mask_crc(crc))
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
