"""Mutable shared-memory channels (reference: python/ray/experimental/channel/
{shared_memory_channel.py,common.py}; C++ side src/ray/core_worker/
experimental_mutable_object_manager.cc).

A ``Channel`` is one writer and ``num_readers`` readers exchanging a sequence of values
through a single in-place-overwritten shared-memory buffer (``_core.ShmChannel``: robust
process-shared mutex + condition variables, no polling). A write blocks until every
reader consumed the previous value, so a chain of channels is a bounded pipeline.

Values are serialized with the framework serializer. CUDA tensors travel through the
node's HBM object store (one D2D copy into the arena on the writer's stream, zero-copy
DLPack view on the reader, no host bounce) when ``gpu=True``; the writer frees a value's
HBM sub-objects once all readers consumed it (readers still holding the tensors keep
them alive through their pins). Payloads larger than the buffer transparently grow the
channel: the writer publishes a resize marker naming a larger segment and all readers
follow it.

Segments are anonymous memfds (``_private/shm_segment.py``): readers open them through
``/proc/<creator pid>/fd/<fd>``, and the kernel frees them with the last process holding
one, so a killed driver or actor leaves nothing in ``/dev/shm``.
"""

from __future__ import annotations

import os
import uuid

from ray_amd._native import _core
from ray_amd._private import shm_segment
from ray_amd.exceptions import RayChannelError, RayChannelTimeoutError

ChannelClosedError = _core.ChannelClosedError
_RESIZE = b"RSZ!"
DEFAULT_BUFFER = 1 << 20


def _shm_dir():
    return "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"


def _to(timeout):
    return -1.0 if timeout is None else max(0.0, float(timeout))


class Channel:
    """Writer/reader endpoints of one channel. Pickling a Channel hands the receiver
    an attached endpoint (same file); only the creating process unlinks it."""

    def __init__(self, num_readers: int = 1, buffer_size_bytes: int = DEFAULT_BUFFER, *,
                 gpu: bool = False, _path: str | None = None):
        self.num_readers = int(num_readers)
        self.gpu = gpu
        self._owner = _path is None
        self._created = []  # (path, memfd or None) of every segment this endpoint created
        if self._owner:
            self.path = self._new_segment(
                os.path.join(_shm_dir(), f"ramd_ch_{os.getpid()}_{uuid.uuid4().hex[:16]}"))
        else:
            self.path = _path
        self._c = _core.ShmChannel(self.path, int(buffer_size_bytes), self.num_readers,
                                   True) if self._owner else None
        self._prev_gpu_oid = None
        self._resizes = 0

    def _new_segment(self, name):
        path, fd = shm_segment.create(name)
        self._created.append((path, fd))
        return path

    def __reduce__(self):
        return (_attach, (self.path, self.num_readers, self.gpu))

    def _chan(self):
        if self._c is None:
            self._c = _core.ShmChannel(self.path)
        return self._c

    # ------------------------------------------------------------------ writer
    def write(self, value, timeout=None, *, _error: bool = False) -> None:
        from ray_amd._private import serialization as ser

        oid = None
        if _error:
            so = ser.serialize_error(value)
        else:
            if self.gpu:
                oid = b"ch" + uuid.uuid4().bytes
            so = ser.serialize(value, object_id=oid)
        data = so.to_bytes()
        self.write_bytes(data, timeout)
        # every reader consumed the previous value before this write went through
        self._free_gpu(self._prev_gpu_oid)
        self._prev_gpu_oid = oid if so.gpu else None

    def write_bytes(self, data, timeout=None) -> None:
        c = self._chan()
        if len(data) > c.capacity:
            c = self._grow(len(data), timeout)
        try:
            ok = c.write(data, _to(timeout))
        except ChannelClosedError:
            raise RayChannelError(f"channel {self.path} is closed") from None
        if not ok:
            raise RayChannelTimeoutError(f"write to channel {self.path} timed out after "
                                         f"{timeout}s (readers did not consume)")

    def _grow(self, need: int, timeout):
        self._resizes += 1
        new_path = self._new_segment(
            os.path.join(_shm_dir(), f"ramd_ch_{os.getpid()}_{uuid.uuid4().hex[:16]}"
                                     f".r{self._resizes}"))
        cap = max(need * 2, self._chan().capacity * 2)
        new = _core.ShmChannel(new_path, cap, self._chan().num_readers, True)
        if not self._chan().write(_RESIZE + new_path.encode(), _to(timeout)):
            raise RayChannelTimeoutError(f"resize of channel {self.path} timed out")
        if self._owner and not shm_segment.is_anonymous(self.path):
            try:
                os.unlink(self.path)  # readers keep their mapping until they switch
            except OSError:
                pass
            self._created = [c for c in self._created if c[0] != self.path]
        self.path = new_path
        self._c = new
        return new

    @staticmethod
    def _free_gpu(oid):
        if oid is None:
            return
        from ray_amd._private import gpu_object_store as gos

        cw = gos._cw()
        if cw is not None:
            gos.free_sub_objects(cw.store.store, oid)

    # ------------------------------------------------------------------ reader
    def read_bytes(self, reader: int = 0, timeout=None) -> bytes:
        while True:
            try:
                b = self._chan().read(reader, _to(timeout))
            except ChannelClosedError:
                raise RayChannelError(f"channel {self.path} is closed") from None
            if b is None:
                raise RayChannelTimeoutError(f"read from channel {self.path} timed out after "
                                             f"{timeout}s")
            if b[:4] == _RESIZE:
                self.path = b[4:].decode()
                self._c = _core.ShmChannel(self.path)
                continue
            return b

    def read(self, reader: int = 0, timeout=None):
        """Returns the next value; a written error is raised."""
        kind, value = self.read_raw(reader, timeout)
        if kind == _KIND_ERROR:
            from ray_amd.exceptions import RayTaskError

            if isinstance(value, RayTaskError):
                raise value.as_instanceof_cause()
            raise value
        return value

    def read_raw(self, reader: int = 0, timeout=None):
        from ray_amd._private import serialization as ser

        return ser.deserialize(memoryview(self.read_bytes(reader, timeout)))

    # ------------------------------------------------------------------ lifecycle
    def close(self) -> None:
        try:
            self._chan().close()
        except Exception:  # noqa: BLE001
            pass

    @property
    def closed(self) -> bool:
        return self._chan().closed

    def destroy(self) -> None:
        """Close and unlink every file this endpoint created."""
        self.close()
        self._free_gpu(self._prev_gpu_oid)
        self._prev_gpu_oid = None
        for p, fd in self._created:
            shm_segment.release(p, fd)
        self._created = []


def _attach(path, num_readers, gpu):
    return Channel(num_readers, gpu=gpu, _path=path)


class ReaderInterface:
    """A bound reader endpoint (reference: ReaderInterface in common.py)."""

    def __init__(self, channel: Channel, reader_index: int):
        self.channel = channel
        self.index = reader_index

    def read(self, timeout=None):
        return self.channel.read(self.index, timeout)


class WriterInterface:
    def __init__(self, channel: Channel):
        self.channel = channel

    def write(self, value, timeout=None):
        self.channel.write(value, timeout)


_KIND_ERROR = 1

__all__ = ["Channel", "ChannelClosedError", "ReaderInterface", "WriterInterface"]
