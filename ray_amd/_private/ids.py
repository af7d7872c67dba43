"""Binary IDs (reference: src/ray/common/id.h, python/ray/includes/unique_ids.pxi).

ObjectID is 20 bytes: 16-byte task id + 4-byte little-endian return/put index, so the
return objects of a task are derivable from its task id (owner never needs a lookup).
"""

from __future__ import annotations

import struct

from ray_amd._native import _core

OBJECT_ID_SIZE = 20
TASK_ID_SIZE = 16


def random_bytes(n: int) -> bytes:
    return _core.random_id(n)


class BaseID:
    __slots__ = ("_b",)
    SIZE = 16

    def __init__(self, b: bytes):
        if len(b) != self.SIZE:
            raise ValueError(f"{type(self).__name__} needs {self.SIZE} bytes, got {len(b)}")
        self._b = b

    @classmethod
    def from_random(cls):
        return cls(random_bytes(cls.SIZE))

    @classmethod
    def from_hex(cls, h: str):
        return cls(bytes.fromhex(h))

    @classmethod
    def nil(cls):
        return cls(b"\xff" * cls.SIZE)

    def is_nil(self):
        return self._b == b"\xff" * self.SIZE

    def binary(self) -> bytes:
        return self._b

    def hex(self) -> str:
        return self._b.hex()

    def __hash__(self):
        return hash(self._b)

    def __eq__(self, o):
        return type(o) is type(self) and o._b == self._b

    def __repr__(self):
        return f"{type(self).__name__}({self.hex()})"

    def __reduce__(self):
        return (type(self), (self._b,))


class JobID(BaseID):
    SIZE = 4

    @classmethod
    def from_int(cls, i: int):
        return cls(struct.pack("<I", i))

    def int(self) -> int:
        return struct.unpack("<I", self._b)[0]


class TaskID(BaseID):
    SIZE = 16


class ActorID(BaseID):
    SIZE = 16


class NodeID(BaseID):
    SIZE = 16


class WorkerID(BaseID):
    SIZE = 16


class PlacementGroupID(BaseID):
    SIZE = 16


class FunctionID(BaseID):
    SIZE = 16


class UniqueID(BaseID):
    SIZE = 16


class ActorClassID(BaseID):
    SIZE = 16


class ObjectID(BaseID):
    """20 bytes: the creating task's id + a 4-byte return / put index."""

    SIZE = OBJECT_ID_SIZE

    def task_id(self) -> TaskID:
        return TaskID(self._b[:TASK_ID_SIZE])


def object_id_for_return(task_id: bytes, index: int) -> bytes:
    return task_id + struct.pack("<I", index)


def object_id_for_put(task_id: bytes, put_index: int) -> bytes:
    return task_id + struct.pack("<I", 0x80000000 | put_index)


def object_index(oid: bytes) -> int:
    return struct.unpack("<I", oid[16:])[0]


def task_id_of(oid: bytes) -> bytes:
    return oid[:16]
