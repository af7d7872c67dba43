"""TFRecord files of ``tf.train.Example`` protos without TensorFlow (reference:
python/ray/data/datasource/tfrecords_datasource.py, tfrecords_datasink.py).

Framing (length, masked CRC32C of the length, payload, masked CRC32C of the payload) is
done by the native core (``_core.tfrecord_index`` / ``tfrecord_encode``: SSE4.2 CRC32C);
the Example protos are encoded and decoded here straight from the protobuf wire format:

    Example  { Features features = 1; }
    Features { map<string, Feature> feature = 1; }        (entries: key = 1, value = 2)
    Feature  { oneof { BytesList bytes_list = 1; FloatList float_list = 2;
                       Int64List int64_list = 3; } }       (each: repeated value = 1)

Row semantics follow the reference: ``bytes`` / ``float32`` / ``int64`` values; a column
whose every row holds exactly one value is unwrapped to scalars, otherwise rows are lists;
``str`` values are written as UTF-8 bytes."""

from __future__ import annotations

import gzip
import os
import struct
from typing import Dict, List, Tuple

import numpy as np

import ray_amd as ray

_BYTES, _FLOAT, _INT = 1, 2, 3


# ------------------------------------------------------------------ wire primitives
def _varint(n: int) -> bytes:
    n &= (1 << 64) - 1  # negative int64 -> 10-byte two's complement varint
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf, pos: int) -> Tuple[int, int]:
    shift = result = 0
    while True:
        b = buf[pos]
        pos += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, pos
        shift += 7
        if shift > 70:
            raise ValueError("malformed varint")


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def _fields(buf, start: int = 0, end: int | None = None):
    """Yield (field_number, wire_type, value) over a message; value is an int for varint /
    fixed fields and a (start, end) span for length-delimited ones."""
    pos = start
    end = len(buf) if end is None else end
    while pos < end:
        key, pos = _read_varint(buf, pos)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v = (pos, pos + n)
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield fn, wt, v


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v


# ------------------------------------------------------------------ Example codec
def decode_example(buf) -> Dict[str, Tuple[int, list]]:
    """Serialized Example -> {feature name: (kind, values)}; kind 0 = empty feature."""
    out: Dict[str, Tuple[int, list]] = {}
    for fn, wt, span in _fields(buf):
        if fn != 1 or wt != 2:
            continue
        for efn, ewt, espan in _fields(buf, *span):  # Features.feature map entries
            if efn != 1 or ewt != 2:
                continue
            name, feat = None, None
            for kfn, _, kspan in _fields(buf, *espan):
                if kfn == 1:
                    name = bytes(buf[kspan[0]:kspan[1]]).decode()
                elif kfn == 2:
                    feat = kspan
            kind, vals = 0, []
            if feat is not None:
                for ffn, _, lspan in _fields(buf, *feat):  # the oneof list
                    kind = ffn
                    for vfn, vwt, v in _fields(buf, *lspan):
                        if vfn != 1:
                            continue
                        if ffn == _BYTES:
                            vals.append(bytes(buf[v[0]:v[1]]))
                        elif ffn == _FLOAT:
                            if vwt == 2:
                                vals.extend(np.frombuffer(bytes(buf[v[0]:v[1]]), "<f4")
                                            .tolist())
                            else:
                                vals.append(struct.unpack("<f", struct.pack("<I", v))[0])
                        elif ffn == _INT:
                            if vwt == 2:
                                p = v[0]
                                while p < v[1]:
                                    x, p = _read_varint(buf, p)
                                    vals.append(_signed64(x))
                            else:
                                vals.append(_signed64(v))
            out[name] = (kind, vals)
    return out


def _feature(value) -> bytes:
    if isinstance(value, np.ndarray):
        value = value.tolist()
    vals = list(value) if isinstance(value, (list, tuple)) else \
        ([] if value is None else [value])
    kinds = set()
    for v in vals:
        if isinstance(v, (bool, np.bool_)) or isinstance(v, (int, np.integer)):
            kinds.add(_INT)
        elif isinstance(v, (float, np.floating)):
            kinds.add(_FLOAT)
        elif isinstance(v, (bytes, bytearray, memoryview, str)):
            kinds.add(_BYTES)
        else:
            raise ValueError(f"Value {v!r} of type {type(v).__name__} cannot be stored in a "
                             f"tf.train.Feature (bytes, float or int)")
    if kinds == {_INT, _FLOAT}:
        kinds = {_FLOAT}
    if len(kinds) > 1:
        raise ValueError(f"mixed value types in one feature: {vals!r}")
    kind = kinds.pop() if kinds else None
    if kind is None:
        raise ValueError("Unable to infer type from partially missing column (an empty or "
                         "null value with no typed rows to take the type from)")
    if kind == _INT:
        body = _ld(1, b"".join(_varint(int(v)) for v in vals))
    elif kind == _FLOAT:
        body = _ld(1, np.asarray(vals, dtype="<f4").tobytes())
    else:
        body = b"".join(_ld(1, v.encode() if isinstance(v, str) else bytes(v)) for v in vals)
    return _ld(kind, body)


def encode_example(row: dict, kinds: Dict[str, int] | None = None) -> bytes:
    entries = []
    for name, value in row.items():
        empty = value is None or (isinstance(value, (list, tuple, np.ndarray)) and
                                  len(value) == 0)
        if empty and kinds and kinds.get(name):
            feat = _ld(kinds[name], b"")  # typed empty list
        else:
            feat = _feature(value)
        entries.append(_ld(1, _ld(1, name.encode()) + _ld(2, feat)))
    return _ld(1, b"".join(entries))


# ------------------------------------------------------------------ file level
def _open_bytes(path: str, compression: str | None) -> bytes:
    with open(path, "rb") as f:
        data = f.read()
    if compression in ("gzip", "GZIP") or (compression is None and path.endswith(".gz")):
        data = gzip.decompress(data)
    elif compression not in (None, "", "none", "NONE"):
        raise ValueError(f"unsupported TFRecord compression {compression!r}")
    return data


def _rows_to_block(rows: List[Dict[str, Tuple[int, list]]]):
    import pyarrow as pa

    names: List[str] = []
    for r in rows:
        for k in r:
            if k not in names:
                names.append(k)
    cols = {}
    for k in names:
        cells = [r.get(k, (0, [])) for r in rows]
        kind = next((c[0] for c in cells if c[0]), 0)
        single = all(len(c[1]) == 1 for c in cells)
        ty = {_BYTES: pa.binary(), _FLOAT: pa.float32(), _INT: pa.int64(), 0: pa.null()}[kind]
        if single:
            cols[k] = pa.array([c[1][0] for c in cells], type=ty)
        else:
            cols[k] = pa.array([c[1] for c in cells], type=pa.list_(ty))
    return pa.table(cols)


def read_file(path: str, verify: bool = True, compression: str | None = None):
    from ray_amd._native import _core

    data = _open_bytes(path, compression)
    mv = memoryview(data)
    rows = [decode_example(mv[o:o + n]) for o, n in _core.tfrecord_index(data, verify)]
    return _rows_to_block(rows)


def encode_block(blk) -> bytes:
    """One block as the bytes of a TFRecord file (framing + CRC32C natively)."""
    from ray_amd._native import _core
    from ray_amd.data import block as B

    kinds = _block_kinds(blk)
    return _core.tfrecord_encode([encode_example(row, kinds) for row in B.to_rows(blk)])


@ray.remote
def _write_tfrecords_block(blk, path, idx, compression):
    from ray_amd._native import _core
    from ray_amd.data import block as B

    kinds = _block_kinds(blk)
    os.makedirs(path, exist_ok=True)
    recs = [encode_example(row, kinds) for row in B.to_rows(blk)]
    data = _core.tfrecord_encode(recs)
    name = f"part_{idx:06d}.tfrecords"
    if compression in ("gzip", "GZIP"):
        data = gzip.compress(data)
        name += ".gz"
    with open(os.path.join(path, name), "wb") as f:
        f.write(data)
    return len(recs)


def _block_kinds(blk) -> Dict[str, int]:
    """Feature kind per column of a (numpy dict) block, so rows whose value is empty still
    write a typed list."""
    out = {}
    for name, col in blk.items():
        arr = np.asarray(col)
        k = arr.dtype.kind
        if k in "iub":
            out[name] = _INT
        elif k == "f":
            out[name] = _FLOAT
        elif k in "SU":
            out[name] = _BYTES
        elif k == "O":
            for v in arr.ravel():
                vals = v.tolist() if isinstance(v, np.ndarray) else v
                vals = vals if isinstance(vals, (list, tuple)) else [vals]
                vals = [x for x in vals if x is not None]
                if vals:
                    x = vals[0]
                    out[name] = _INT if isinstance(x, (int, np.integer)) else \
                        _FLOAT if isinstance(x, (float, np.floating)) else _BYTES
                    break
    return out
