"""Runtime context (reference: python/ray/runtime_context.py)."""

from __future__ import annotations

import os


class RuntimeContext:
    def __init__(self, worker):
        self._w = worker

    @property
    def _cw(self):
        return self._w.core

    def get_job_id(self) -> str:
        from ray_amd._private.ids import JobID

        return JobID.from_int(self._cw.job_id or 0).hex()

    @property
    def job_id(self):
        from ray_amd._private.ids import JobID

        return JobID.from_int(self._cw.job_id or 0)

    def get_node_id(self) -> str:
        return self._cw.node_id.hex()

    @property
    def node_id(self):
        from ray_amd._private.ids import NodeID

        return NodeID(self._cw.node_id)

    def get_worker_id(self) -> str:
        return self._cw.worker_id.hex()

    def get_task_id(self):
        t = getattr(self._cw.current_task, "tid", None)
        return t.hex() if t else None

    def get_task_name(self):
        """The current task's name (``options(name=...)`` or the function / method)."""
        spec = getattr(self._cw.current_task, "spec", None)
        if not spec:
            return None
        m = spec.get("method")
        if m and spec.get("name") in (None, m):  # actor call: "Class.method"
            inst = self._cw.actor_instance
            return f"{type(inst).__name__}.{m}" if inst is not None else m
        return spec.get("name") or m

    def get_task_function_name(self):
        """Fully qualified name of the function (or ``Class.method``) being executed."""
        spec = getattr(self._cw.current_task, "spec", None)
        if not spec:
            return None
        if spec.get("method"):
            inst = self._cw.actor_instance
            cls = type(inst) if inst is not None else None
            qual = f"{cls.__module__}.{cls.__qualname__}" if cls else "actor"
            return f"{qual}.{spec['method']}"
        fn = self._cw._load_function(spec["fn"]) if spec.get("fn") is not None else None
        if fn is None:
            return spec.get("name")
        return f"{getattr(fn, '__module__', '')}.{getattr(fn, '__qualname__', fn)}"

    def get(self):
        """Deprecated dict form of the context (reference: RuntimeContext.get)."""
        return {"job_id": self.get_job_id(), "node_id": self.get_node_id(),
                "namespace": self.namespace, "task_id": self.get_task_id(),
                "actor_id": self.get_actor_id()}

    def get_actor_id(self):
        a = self._cw.actor_id
        return a.hex() if a else None

    @property
    def actor_id(self):
        from ray_amd._private.ids import ActorID

        a = self._cw.actor_id
        return ActorID(a) if a else None

    def get_actor_name(self):
        spec = self._cw.actor_spec
        return None if spec is None else spec.get("actor_name")

    @property
    def namespace(self):
        return self._cw.namespace

    def get_placement_group_id(self):
        from ray_amd.util.placement_group import get_current_placement_group

        pg = get_current_placement_group()
        return pg.id.hex() if pg else None

    @property
    def current_placement_group_id(self):
        from ray_amd.util.placement_group import get_current_placement_group

        pg = get_current_placement_group()
        return pg.id if pg else None

    @property
    def should_capture_child_tasks_in_placement_group(self):
        spec = getattr(self._cw.current_task, "spec", None) or self._cw.actor_spec
        st = (spec or {}).get("strategy")
        return bool(isinstance(st, dict) and st.get("capture"))

    def get_assigned_resources(self):
        spec = getattr(self._cw.current_task, "spec", None) or self._cw.actor_spec
        return dict((spec or {}).get("resources") or {})

    @property
    def task_id(self):
        """Deprecated property form of ``get_task_id``."""
        return self.get_task_id()

    def get_resource_ids(self):
        """Deprecated: ``{"GPU": [(id, fraction), ...]}`` of this worker."""
        res = self.get_assigned_resources()
        frac = float(res.get("GPU", 1.0) or 1.0)
        return {"GPU": [(int(i), frac) for i in self._cw.gpu_ids]}

    def get_accelerator_ids(self):
        return {"GPU": [str(i) for i in self._cw.gpu_ids]}

    def get_runtime_env_string(self):
        import json

        return json.dumps(self._w.runtime_env or {})

    @property
    def runtime_env(self):
        return dict(self._w.runtime_env or {})

    @property
    def gcs_address(self):
        return self._w.session_dir

    def was_current_actor_reconstructed(self):
        return bool(os.environ.get("RAY_AMD_ACTOR_RESTARTED"))

    @property
    def current_actor(self):
        from ray_amd.actor import ActorHandle

        cw = self._cw
        if cw.actor_id is None:
            raise RuntimeError("This method is only available in an actor.")
        spec = cw.actor_spec
        return ActorHandle(cw.actor_id, spec.get("name"), spec.get("method_meta"), spec["owner"])


def get_runtime_context() -> RuntimeContext:
    from ray_amd._private import worker as W

    W._check_connected()
    return RuntimeContext(W.global_worker)
