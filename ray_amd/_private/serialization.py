"""Object serialization (reference: python/ray/_private/serialization.py).

Format of a serialized object (identical inline — bytes inside a message — and
in the shared-memory store, so an inline value can be promoted to the store by
a plain memcpy):

    u8 magic | u8 kind | u16 nbuf | u32 pad | u64 inband_len | nbuf x (u64 off, u64 len)
    inband pickle bytes ... | 64-byte aligned out-of-band buffers ...

Pickle protocol 5 with out-of-band buffers: numpy arrays and CPU torch tensors
are written once, straight into the store, and come back as zero-copy views of
the shared segment. CUDA tensors are routed to the HBM object store (see
``ray_amd._private.gpu_object_store``): only a descriptor is pickled.
"""

from __future__ import annotations

import copyreg
import io
import pickle
import struct
import sys
import threading

import cloudpickle

KIND_PICKLE = 0
KIND_ERROR = 1
KIND_RAW = 2
KIND_ACTOR_HANDLE = 3

_MAGIC = 0xA5
_HDR = struct.Struct("<BBHIQ")
_BUF = struct.Struct("<QQ")
ALIGN = 64

_custom_reducers: dict = {}
_tls = threading.local()


def _ctx():
    c = getattr(_tls, "ctx", None)
    return c


class _SerContext:
    __slots__ = ("refs", "gpu", "object_id")

    def __init__(self, object_id=None):
        self.refs = []
        self.gpu = []
        self.object_id = object_id


def current_context():
    return getattr(_tls, "ctx", None)


def register_serializer(cls, *, serializer, deserializer):
    """ray.util.register_serializer parity."""

    def reducer(obj):
        return (_call_deserializer, (deserializer, serializer(obj)))

    _custom_reducers[cls] = reducer


def deregister_serializer(cls):
    _custom_reducers.pop(cls, None)


def _call_deserializer(fn, payload):
    return fn(payload)


# ----------------------------------------------------------------------------- torch
def _torch_reduce(t):
    import torch

    if t.is_cuda:
        from ray_amd._private import gpu_object_store as gos

        red = gos.reduce_cuda_tensor(t)
        if red is not None:
            return red
        return (_rebuild_cpu_to_cuda, (_torch_reduce(t.detach().cpu()), t.device.index))
    if t.requires_grad or t.is_sparse or t.is_quantized or not t.is_contiguous() or \
            t.layout != torch.strided:
        return t.__reduce_ex__(2)
    dt = t.dtype
    shape = tuple(t.shape)
    if dt == torch.bfloat16:
        arr = t.view(torch.int16).numpy()
    elif dt in (torch.float8_e4m3fn, torch.float8_e5m2) if hasattr(torch, "float8_e4m3fn") \
            else False:
        arr = t.view(torch.uint8).numpy()
    else:
        try:
            arr = t.numpy()
        except Exception:
            return t.__reduce_ex__(2)
    return (_rebuild_cpu_tensor, (pickle.PickleBuffer(arr) if arr.size else arr.tobytes(),
                                  str(dt), shape, arr.dtype.str))


def _rebuild_cpu_tensor(buf, dtype_s, shape, np_dtype):
    import numpy as np
    import torch

    arr = np.frombuffer(buf, dtype=np.dtype(np_dtype)).reshape(shape)
    if not arr.flags.writeable:
        # views of sealed shm objects are read-only; torch needs a writable array
        arr = arr.copy() if arr.nbytes < (1 << 16) else _writable_view(arr)
    t = torch.from_numpy(arr)
    dt = getattr(torch, dtype_s.replace("torch.", ""))
    if t.dtype != dt:
        t = t.view(dt)
    return t


def _writable_view(arr):
    import numpy as np

    try:
        arr.setflags(write=True)
        return arr
    except ValueError:
        # underlying buffer is a read-only memoryview of a sealed object; the
        # object is immutable by contract, so mirror Ray (which hands out
        # read-only numpy) but torch requires writable: fall back to a copy.
        return np.array(arr, copy=True)


def _rebuild_cpu_to_cuda(cpu_reduced, device):
    fn, args = cpu_reduced
    t = fn(*args) if callable(fn) else None
    return t.to(f"cuda:{device}")


class _Pickler(cloudpickle.CloudPickler):
    def reducer_override(self, obj):
        t = type(obj)
        r = _custom_reducers.get(t)
        if r is not None:
            return r(obj)
        if t.__module__ == "torch" and t.__name__ in ("Tensor", "Parameter") and \
                "torch" in sys.modules:
            return _torch_reduce(obj)
        return super().reducer_override(obj)


class SerializedObject:
    __slots__ = ("kind", "inband", "buffers", "refs", "gpu", "_layout", "total")

    def __init__(self, kind, inband, buffers=(), refs=(), gpu=()):
        self.kind = kind
        self.inband = inband
        self.buffers = [b.raw() if isinstance(b, pickle.PickleBuffer) else memoryview(b)
                        for b in buffers]
        self.refs = list(refs)
        self.gpu = list(gpu)
        hdr = _HDR.size + _BUF.size * len(self.buffers)
        off = hdr + len(inband)
        layout = []
        for b in self.buffers:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            layout.append((off, b.nbytes))
            off += b.nbytes
        self._layout = layout
        self.total = off

    def write_to(self, mv, big_copy=None) -> None:
        """Lay the object out in `mv`. big_copy(offset, buffer), if given, moves the
        out-of-band buffers of 16 MiB and more (the store's multi-threaded copy)."""
        _HDR.pack_into(mv, 0, _MAGIC, self.kind, len(self.buffers), 0, len(self.inband))
        p = _HDR.size
        for off, n in self._layout:
            _BUF.pack_into(mv, p, off, n)
            p += _BUF.size
        mv[p:p + len(self.inband)] = self.inband
        for (off, n), b in zip(self._layout, self.buffers):
            if n:
                if big_copy is not None and n >= (16 << 20) and b.c_contiguous:
                    big_copy(off, b)
                else:
                    mv[off:off + n] = b.cast("B") if b.format != "B" or b.ndim != 1 else b

    def to_bytes(self) -> bytes:
        if not self.buffers:
            return _HDR.pack(_MAGIC, self.kind, 0, 0, len(self.inband)) + self.inband
        ba = bytearray(self.total)
        self.write_to(memoryview(ba))
        return bytes(ba)


def serialize(value, object_id=None) -> SerializedObject:
    """Serialize a Python value; records contained ObjectRefs and GPU tensors."""
    if type(value) is bytes and len(value) > 4096:
        return SerializedObject(KIND_RAW, b"", [value])
    ctx = _SerContext(object_id)
    prev = getattr(_tls, "ctx", None)
    _tls.ctx = ctx
    buffers = []
    try:
        t = type(value)
        if t in (int, float, str, bool, type(None)) or (t is bytes and len(value) <= 4096):
            inband = pickle.dumps(value, protocol=5)
        else:
            f = io.BytesIO()
            p = _Pickler(f, protocol=5, buffer_callback=buffers.append)
            p.dump(value)
            inband = f.getvalue()
    finally:
        _tls.ctx = prev
    return SerializedObject(KIND_PICKLE, inband, buffers, ctx.refs, ctx.gpu)


def serialize_error(exc) -> SerializedObject:
    try:
        inband = cloudpickle.dumps(exc, protocol=5)
    except Exception:
        from ray_amd.exceptions import RayTaskError

        inband = cloudpickle.dumps(RayTaskError("<unknown>", repr(exc), RuntimeError(repr(exc))))
    return SerializedObject(KIND_ERROR, inband)


class DeserializeContext:
    __slots__ = ("anchor", "source_pin")

    def __init__(self, anchor=None, source_pin=None):
        self.anchor = anchor  # address of the process keeping contained refs alive
        self.source_pin = source_pin


_dtls = threading.local()


def current_deser_context():
    return getattr(_dtls, "ctx", None)


def header(mv):
    magic, kind, nbuf, _, inband_len = _HDR.unpack_from(mv, 0)
    if magic != _MAGIC:
        raise ValueError("corrupt serialized object")
    return kind, nbuf, inband_len


def deserialize(mv, ctx: DeserializeContext | None = None):
    """Deserialize from a memoryview (zero-copy for out-of-band buffers).

    Returns (kind, value). For KIND_ERROR the value is the exception instance."""
    if not isinstance(mv, memoryview):
        mv = memoryview(mv)
    magic, kind, nbuf, _, inband_len = _HDR.unpack_from(mv, 0)
    if magic != _MAGIC:
        raise ValueError("corrupt serialized object")
    p = _HDR.size
    bufs = []
    for _ in range(nbuf):
        off, n = _BUF.unpack_from(mv, p)
        p += _BUF.size
        bufs.append(mv[off:off + n])
    inband = mv[p:p + inband_len]
    if kind == KIND_RAW:
        return kind, bytes(bufs[0])
    prev = getattr(_dtls, "ctx", None)
    _dtls.ctx = ctx
    try:
        value = pickle.loads(inband, buffers=bufs)
    finally:
        _dtls.ctx = prev
    return kind, value


copyreg  # noqa: B018  (kept for API parity imports)
