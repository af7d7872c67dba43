"""ObjectRef (reference: python/ray/includes/object_ref.pxi).

Creating/deleting an ObjectRef adjusts the process-local reference count held by
the CoreWorker; pickling one records it in the active serialization context so
the owner can track borrowers (distributed reference counting)."""

from __future__ import annotations

import asyncio
import concurrent.futures

from ray_amd._private import serialization as _ser


def _cw():
    from ray_amd._private import worker as _w

    return _w.global_worker.core


class ObjectRef:
    __slots__ = ("_id", "_owner", "_cw", "__weakref__")

    def __init__(self, oid: bytes, owner: str, *, _add_ref: bool = True, _cw_obj=None):
        self._id = oid
        self._owner = owner
        cw = _cw_obj if _cw_obj is not None else _cw()
        self._cw = cw
        if _add_ref and cw is not None:
            cw.add_local_ref(oid, owner)

    def binary(self) -> bytes:
        return self._id

    def hex(self) -> str:
        return self._id.hex()

    def task_id(self):
        from ray_amd._private.ids import TaskID

        return TaskID(self._id[:16])

    def owner_address(self) -> str:
        return self._owner

    def __repr__(self):
        return f"ObjectRef({self._id.hex()})"

    def __hash__(self):
        return hash(self._id)

    def __eq__(self, other):
        return isinstance(other, ObjectRef) and other._id == self._id

    def __del__(self):
        cw = self._cw
        if cw is not None:
            try:
                cw.remove_local_ref(self._id)
            except Exception:
                pass

    def __reduce__(self):
        ctx = _ser.current_context()
        if ctx is not None:
            ctx.refs.append(self)
        return (_rebuild_ref, (self._id, self._owner))

    # ---- futures / asyncio
    def __class_getitem__(cls, item):  # ObjectRef[int] in annotations
        return cls

    def future(self) -> concurrent.futures.Future:
        return self._cw.as_concurrent_future(self)

    def __await__(self):
        return self._as_asyncio_future().__await__()

    def _as_asyncio_future(self):
        return asyncio.wrap_future(self.future())

    def is_nil(self):
        return self._id == b"\xff" * 20

    @classmethod
    def nil(cls):
        return cls(b"\xff" * 20, "", _add_ref=False)


def _rebuild_ref(oid, owner):
    cw = _cw()
    ref = ObjectRef(oid, owner, _add_ref=False, _cw_obj=cw)
    if cw is not None:
        cw.add_local_ref(oid, owner, deserialized=True)
    return ref


class ObjectRefGenerator:
    """Streaming generator of ObjectRefs (reference: _raylet.pyx ObjectRefGenerator).

    Items arrive as the executing task yields them; iteration blocks until the
    next item is reported or the task finishes."""

    def __init__(self, task_id: bytes, cw, owner: str):
        self._task_id = task_id
        self._cw = cw
        self._owner = owner
        self._index = 0

    def __iter__(self):
        return self

    def __next__(self):
        ref = self._cw.next_stream_item(self._task_id, self._index, None)
        if ref is None:
            raise StopIteration
        self._index += 1
        return ref

    def __aiter__(self):
        return self

    async def __anext__(self):
        loop = asyncio.get_running_loop()
        ref = await loop.run_in_executor(None, self._cw.next_stream_item, self._task_id,
                                         self._index, None)
        if ref is None:
            raise StopAsyncIteration
        self._index += 1
        return ref

    def completed(self):
        return self._cw.stream_completed_ref(self._task_id)

    def __del__(self):
        try:
            self._cw.drop_stream(self._task_id)
        except Exception:
            pass


# Reference name for dynamic generators
DynamicObjectRefGenerator = ObjectRefGenerator
