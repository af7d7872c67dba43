"""Avro object container files (reference: python/ray/data/datasource/avro_datasource.py,
which reads through fastavro — not installed here, so the format is decoded directly).

Container layout (Avro 1.11 spec): magic ``Obj\\x01``, a metadata map (``avro.schema``
JSON, ``avro.codec`` = ``null`` or ``deflate``), a 16-byte sync marker, then blocks of
``(record count, byte size, records, sync)``. Binary encoding: int/long as zig-zag
varints, float/double little-endian IEEE, bytes/string length-prefixed, arrays/maps as
counted blocks (a negative count carries a byte size), unions as a branch index.
Supported schema types: the primitives, record, enum, array, map, union, fixed, and the
logical types as their underlying values. ``write_ocf`` writes the same format (tests and
round trips)."""

from __future__ import annotations

import io
import json
import os
import struct
import zlib
from typing import Any, List

MAGIC = b"Obj\x01"


class _Reader:
    __slots__ = ("buf", "pos")

    def __init__(self, buf: bytes, pos: int = 0):
        self.buf, self.pos = buf, pos

    def long(self) -> int:
        shift = result = 0
        buf = self.buf
        while True:
            b = buf[self.pos]
            self.pos += 1
            result |= (b & 0x7F) << shift
            if not b & 0x80:
                return (result >> 1) ^ -(result & 1)
            shift += 7

    def take(self, n: int) -> bytes:
        out = self.buf[self.pos:self.pos + n]
        if len(out) != n:
            raise ValueError("truncated Avro data")
        self.pos += n
        return out


def _named(schema, names: dict):
    if isinstance(schema, str) and schema in names:
        return names[schema]
    return schema


def _register(schema, names: dict, ns: str = ""):
    """Collect named types (record/enum/fixed) so later references by name resolve."""
    if isinstance(schema, list):
        for s in schema:
            _register(s, names, ns)
    elif isinstance(schema, dict):
        t = schema.get("type")
        if t in ("record", "error", "enum", "fixed"):
            name = schema["name"]
            space = schema.get("namespace", ns)
            names[name] = schema
            if space and "." not in name:
                names[f"{space}.{name}"] = schema
            for f in schema.get("fields", ()):
                _register(f["type"], names, space)
        elif t == "array":
            _register(schema["items"], names, ns)
        elif t == "map":
            _register(schema["values"], names, ns)


def _decode(r: _Reader, schema, names: dict) -> Any:
    schema = _named(schema, names)
    if isinstance(schema, list):  # union
        return _decode(r, schema[r.long()], names)
    t = schema["type"] if isinstance(schema, dict) else schema
    if isinstance(t, (dict, list)):
        return _decode(r, t, names)
    if t == "null":
        return None
    if t == "boolean":
        return r.take(1) != b"\x00"
    if t in ("int", "long"):
        return r.long()
    if t == "float":
        return struct.unpack("<f", r.take(4))[0]
    if t == "double":
        return struct.unpack("<d", r.take(8))[0]
    if t == "bytes":
        return bytes(r.take(r.long()))
    if t == "string":
        return r.take(r.long()).decode("utf-8")
    if t == "fixed":
        return bytes(r.take(schema["size"]))
    if t == "enum":
        return schema["symbols"][r.long()]
    if t in ("record", "error"):
        return {f["name"]: _decode(r, f["type"], names) for f in schema["fields"]}
    if t in ("array", "map"):
        out = [] if t == "array" else {}
        while True:
            n = r.long()
            if n == 0:
                return out
            if n < 0:
                n = -n
                r.long()  # block byte size
            for _ in range(n):
                if t == "array":
                    out.append(_decode(r, schema["items"], names))
                else:
                    k = r.take(r.long()).decode("utf-8")
                    out[k] = _decode(r, schema["values"], names)
    if isinstance(t, str) and t in names:
        return _decode(r, names[t], names)
    raise ValueError(f"unsupported Avro type {t!r}")


def read_ocf(data: bytes) -> tuple[dict, List[Any]]:
    """(schema, records) of one Avro object container file."""
    if data[:4] != MAGIC:
        raise ValueError("not an Avro object container file (bad magic)")
    r = _Reader(data, 4)
    meta = _decode(r, {"type": "map", "values": "bytes"}, {})
    sync = r.take(16)
    schema = json.loads(meta["avro.schema"].decode())
    codec = meta.get("avro.codec", b"null").decode()
    names: dict = {}
    _register(schema, names)
    records = []
    while r.pos < len(data):
        count = r.long()
        size = r.long()
        block = r.take(size)
        if codec == "deflate":
            block = zlib.decompress(block, -15)
        elif codec != "null":
            raise ValueError(f"unsupported Avro codec {codec!r} (null and deflate are)")
        br = _Reader(block)
        for _ in range(count):
            records.append(_decode(br, schema, names))
        if r.take(16) != sync:
            raise ValueError("Avro sync marker mismatch (corrupt file)")
    return schema, records


# ------------------------------------------------------------------ writer
def _zz(n: int) -> bytes:
    n = (n << 1) ^ (n >> 63)
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _branch(schema: list, v, names) -> int:
    for i, s in enumerate(schema):
        s = _named(s, names)
        t = s["type"] if isinstance(s, dict) else s
        if v is None and t == "null":
            return i
        if v is None:
            continue
        if (t == "boolean" and isinstance(v, bool)) or \
                (t in ("int", "long") and isinstance(v, int) and not isinstance(v, bool)) or \
                (t in ("float", "double") and isinstance(v, (int, float))
                 and not isinstance(v, bool)) or \
                (t == "string" and isinstance(v, str)) or \
                (t in ("bytes", "fixed") and isinstance(v, (bytes, bytearray))) or \
                (t in ("record", "map") and isinstance(v, dict)) or \
                (t == "array" and isinstance(v, (list, tuple))) or \
                (t == "enum" and isinstance(v, str)):
            return i
    raise ValueError(f"value {v!r} matches no branch of union {schema}")


def _encode(out: io.BytesIO, schema, v, names: dict) -> None:
    schema = _named(schema, names)
    if isinstance(schema, list):
        i = _branch(schema, v, names)
        out.write(_zz(i))
        return _encode(out, schema[i], v, names)
    t = schema["type"] if isinstance(schema, dict) else schema
    if isinstance(t, (dict, list)):
        return _encode(out, t, v, names)
    if t == "null":
        return
    if t == "boolean":
        out.write(b"\x01" if v else b"\x00")
    elif t in ("int", "long"):
        out.write(_zz(int(v)))
    elif t == "float":
        out.write(struct.pack("<f", v))
    elif t == "double":
        out.write(struct.pack("<d", v))
    elif t in ("bytes", "string"):
        b = v.encode("utf-8") if isinstance(v, str) else bytes(v)
        out.write(_zz(len(b)))
        out.write(b)
    elif t == "fixed":
        out.write(bytes(v))
    elif t == "enum":
        out.write(_zz(schema["symbols"].index(v)))
    elif t in ("record", "error"):
        for f in schema["fields"]:
            _encode(out, f["type"], v.get(f["name"], f.get("default")), names)
    elif t == "array":
        if v:
            out.write(_zz(len(v)))
            for x in v:
                _encode(out, schema["items"], x, names)
        out.write(b"\x00")
    elif t == "map":
        if v:
            out.write(_zz(len(v)))
            for k, x in v.items():
                _encode(out, "string", k, names)
                _encode(out, schema["values"], x, names)
        out.write(b"\x00")
    else:
        raise ValueError(f"unsupported Avro type {t!r}")


def write_ocf(path: str, schema: dict, records, codec: str = "null",
              block_records: int = 1000) -> None:
    names: dict = {}
    _register(schema, names)
    sync = os.urandom(16)
    out = io.BytesIO()
    out.write(MAGIC)
    _encode(out, {"type": "map", "values": "bytes"},
            {"avro.schema": json.dumps(schema).encode(), "avro.codec": codec.encode()}, {})
    out.write(sync)
    records = list(records)
    for s in range(0, len(records), block_records):
        chunk = records[s:s + block_records]
        body = io.BytesIO()
        for rec in chunk:
            _encode(body, schema, rec, names)
        data = body.getvalue()
        if codec == "deflate":
            c = zlib.compressobj(wbits=-15)
            data = c.compress(data) + c.flush()
        elif codec != "null":
            raise ValueError(f"unsupported Avro codec {codec!r}")
        out.write(_zz(len(chunk)))
        out.write(_zz(len(data)))
        out.write(data)
        out.write(sync)
    with open(path, "wb") as f:
        f.write(out.getvalue())


def read_file(path: str):
    import pyarrow as pa

    with open(path, "rb") as f:
        _, records = read_ocf(f.read())
    if not records:
        return {}
    if all(isinstance(r, dict) for r in records):
        return pa.Table.from_pylist(records)
    return pa.table({"value": records})
