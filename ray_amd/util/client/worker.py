"""Client-side core worker (reference: python/ray/util/client/worker.py:Worker)."""

from __future__ import annotations

import collections
import concurrent.futures
import pickle
import threading
from multiprocessing.connection import Client

import cloudpickle

from ray_amd.util.client import common


class ClientCoreWorker:
    """Implements the CoreWorker surface the public API uses, over one TCP link."""

    mode = "client"

    def __init__(self, host: str, port: int, namespace=None, runtime_env=None):
        self.conn = Client((host, int(port)), authkey=common.AUTHKEY)
        self._lock = threading.Lock()
        self.refs: collections.Counter = collections.Counter()
        self.handles: collections.Counter = collections.Counter()
        self.actor_escaped: set = set()
        self._keys: dict = {}
        self._pool = concurrent.futures.ThreadPoolExecutor(4, thread_name_prefix="ray_amd-client")
        self._stopped = False
        info = self._call("init", namespace, runtime_env)
        self.namespace = info["namespace"]
        self.job_id = info["job_id"]
        self.node_id = info["node_id"]
        self.addr = f"ray://{host}:{port}"
        self.gpu_ids = []
        self.local_mode = False
        self.actor_id = None
        self.actor_spec = None
        self.current_task = threading.local()
        self.server_info = info

    # ---------------------------------------------------------------- transport
    def _call(self, op, *args):
        with self._lock:
            self.conn.send_bytes(pickle.dumps((op, args), protocol=5))
            ok, payload = pickle.loads(self.conn.recv_bytes())
        if not ok:
            from ray_amd.exceptions import RayTaskError

            if isinstance(payload, RayTaskError) and hasattr(payload, "as_instanceof_cause"):
                raise payload.as_instanceof_cause()  # `except ValueError` works as locally
            raise payload
        return payload

    def _dumps(self, obj):
        def on_ref(r):
            return ("ref", r._id)

        def on_actor(h):
            return ("actor", h._actor_id)

        return common.dumps(obj, on_ref, on_actor)

    def _loads(self, data):
        from ray_amd.actor import ActorHandle
        from ray_amd.object_ref import ObjectRef

        def load(pid):
            if pid[0] == "ref":
                return ObjectRef(pid[1], self.addr, _cw_obj=self)
            _, aid, cls_name, meta = pid
            return ActorHandle(aid, cls_name, meta, self.addr)

        return common.loads(data, load)

    def _refs(self, oids):
        from ray_amd.object_ref import ObjectRef

        return [ObjectRef(o, self.addr, _cw_obj=self) for o in oids]

    # ---------------------------------------------------------------- ref counting
    def add_local_ref(self, oid, owner, deserialized=False):
        self.refs[oid] += 1

    def remove_local_ref(self, oid):
        self.refs[oid] -= 1
        if self.refs[oid] <= 0:
            del self.refs[oid]
            self._release("release", oid)

    def actor_handle_created(self, aid):
        self.handles[aid] += 1

    def actor_handle_deleted(self, aid, owner=None):
        self.handles[aid] -= 1
        if self.handles[aid] <= 0:
            del self.handles[aid]
            self._release("release_actor", aid)

    def _release(self, op, key):
        if self._stopped:
            return
        try:
            self._call(op, key)
        except Exception:
            pass

    def _subscribe_actor(self, aid):
        pass

    # ---------------------------------------------------------------- API surface
    def export(self, obj) -> str:
        k = self._keys.get(id(obj))
        if k is None:
            k = self._call("export", cloudpickle.dumps(obj))
            self._keys[id(obj)] = k
        return k

    def put_object(self, value):
        return self._refs([self._call("put", self._dumps(value))])[0]

    def get_objects(self, refs, timeout=None):
        return self._loads(self._call("get", [r._id for r in refs], timeout))

    def wait_refs(self, oids, num_returns, timeout):
        return set(self._call("wait", list(oids), num_returns, timeout))

    def _maybe_stream(self, out):
        """A streaming task answers with ("gen", task id): the generator lives in the
        server session and each item is fetched with one round trip."""
        if isinstance(out, tuple) and out and out[0] == "gen":
            from ray_amd.object_ref import ObjectRefGenerator

            return ObjectRefGenerator(out[1], self, self.addr)
        return self._refs(out)

    def submit_task(self, fn_key, args, kwargs, opts, name):
        return self._maybe_stream(self._call("task", fn_key, self._dumps((args, kwargs)), opts,
                                             name))

    def next_stream_item(self, tid, index, timeout):
        oid = self._call("gen_next", tid, index, timeout)
        return None if oid is None else self._refs([oid])[0]

    def stream_completed_ref(self, tid):
        return self._call("gen_done", tid)

    def drop_stream(self, tid):
        self._release("gen_drop", tid)

    def create_actor(self, actor_id, cls_key, args, kwargs, opts, cls_name, meta):
        return self._call("actor", actor_id, cls_key, self._dumps((args, kwargs)), opts,
                          cls_name, meta)

    def submit_actor_task(self, actor_id, method, args, kwargs, opts):
        return self._maybe_stream(self._call("actor_task", actor_id, method,
                                             self._dumps((args, kwargs)), opts))

    def kill_actor(self, actor_id, no_restart=True):
        self._call("kill", actor_id, no_restart)

    def cancel(self, ref, force=False, recursive=True):
        self._call("cancel", ref._id, force, recursive)

    def call_raylet(self, method, *args, timeout=None):
        return self._call("raylet", method, args)

    def as_concurrent_future(self, ref):
        return self._pool.submit(lambda: self.get_objects([ref])[0])

    def _flush_task_events(self):
        pass

    def shutdown(self):
        if self._stopped:
            return
        try:
            self._call("disconnect")
        except Exception:
            pass
        self._stopped = True
        try:
            self.conn.close()
        except Exception:
            pass
        self._pool.shutdown(wait=False)
