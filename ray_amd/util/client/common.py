"""Wire format shared by the Ray Client worker and server."""

from __future__ import annotations

import io
import os
import pickle

import cloudpickle

AUTHKEY = os.environ.get("RAY_AMD_CLIENT_AUTHKEY", "ray_amd_client").encode()


class RefPickler(cloudpickle.Pickler):
    """Pickles ObjectRef / ActorHandle as persistent ids resolved by the peer."""

    def __init__(self, f, on_ref, on_actor):
        super().__init__(f, protocol=5)
        self._on_ref, self._on_actor = on_ref, on_actor

    def persistent_id(self, obj):
        from ray_amd.actor import ActorHandle
        from ray_amd.object_ref import ObjectRef

        if type(obj) is ObjectRef:
            return self._on_ref(obj)
        if type(obj) is ActorHandle:
            return self._on_actor(obj)
        return None


class RefUnpickler(pickle.Unpickler):
    def __init__(self, f, load):
        super().__init__(f)
        self._load = load

    def persistent_load(self, pid):
        return self._load(pid)


def dumps(obj, on_ref, on_actor) -> bytes:
    buf = io.BytesIO()
    RefPickler(buf, on_ref, on_actor).dump(obj)
    return buf.getvalue()


def loads(data: bytes, load):
    return RefUnpickler(io.BytesIO(data), load).load()
