"""Actors (reference: python/ray/actor.py).

An ActorClass exports the user class once; ``.remote()`` registers the actor
with the raylet/GCS, which leases a dedicated worker and runs ``__init__`` there.
Handles submit method calls directly to the actor's worker (ordered per caller).
"""

from __future__ import annotations

import inspect
import weakref

from ray_amd._private import options as _opt


def _cw_key(cw):
    """Cache key of a connection: the worker id (client connections: the object)."""
    return getattr(cw, "worker_id", None) or id(cw)


def _method_meta(cls):
    meta = {}
    is_async = False
    groups = {}
    for name, m in inspect.getmembers(cls):
        if name.startswith("__") and name not in ("__call__",):
            continue
        if not callable(m):
            continue
        fn = m
        o = dict(getattr(fn, "__ray_amd_method_options__", {}) or {})
        if inspect.iscoroutinefunction(fn) or inspect.isasyncgenfunction(fn):
            is_async = True
        if inspect.isgeneratorfunction(fn) or inspect.isasyncgenfunction(fn):
            o.setdefault("num_returns", "streaming")
        if o.get("concurrency_group"):
            groups[name] = o["concurrency_group"]
        meta[name] = o
    meta["__is_async__"] = is_async
    meta["__groups__"] = groups
    return meta


class ActorMethod:
    def __init__(self, handle, name, options):
        self._handle = handle
        self._name = name
        self._options = options

    def remote(self, *args, **kwargs):
        return self._handle._submit(self._name, args, kwargs, self._options)

    def options(self, **opts):
        merged = dict(self._options)
        merged.update(opts)
        return ActorMethod(self._handle, self._name, merged)

    def bind(self, *args, **kwargs):
        from ray_amd.dag import ClassMethodNode

        return ClassMethodNode(self._handle, self._name, args, kwargs, self._options)

    def __call__(self, *a, **k):
        raise TypeError(f"Actor methods cannot be called directly. Instead of running "
                        f"'object.{self._name}()', try 'object.{self._name}.remote()'.")


# key in an ActorHandle's method-metadata dict holding actor-level options that apply to
# every call made through the handle (max_pending_calls, enable_task_events)
_HANDLE_OPTS = "__ray_amd_handle_opts__"


class ActorHandle:
    def __init__(self, actor_id: bytes, class_name: str, meta: dict, owner: str, *,
                 _register=True):
        self._actor_id = actor_id
        self._class_name = class_name
        self._meta = meta or {}
        self._owner = owner
        from ray_amd._private import worker as W

        self._cw = W.global_worker.core
        if _register and self._cw is not None:
            self._cw.actor_handle_created(actor_id)

    @classmethod
    def _from_info(cls, actor_id, class_name, meta, owner):
        return cls(actor_id, class_name, meta, owner)

    @property
    def _ray_actor_id(self):
        from ray_amd._private.ids import ActorID

        return ActorID(self._actor_id)

    def __getattr__(self, name):
        special = ("__ray_terminate__", "__call__", "__ray_call__", "__ray_ready__")
        if name.startswith("_") and name not in special:
            raise AttributeError(name)
        meta = self._meta
        if name not in meta and name not in special and meta:
            raise AttributeError(f"'{self._class_name}' actor has no method '{name}'")
        return ActorMethod(self, name, dict(meta.get(name, {})))

    def _submit(self, name, args, kwargs, opts):
        from ray_amd._private import worker as W

        cw = W._check_connected()
        nret = opts.get("num_returns", 1)
        o = {"num_returns": nret, "name": opts.get("name"),
             "concurrency_group": opts.get("concurrency_group")}
        if "max_task_retries" in opts:
            o["max_task_retries"] = opts["max_task_retries"]
        # actor-level options the handle carries (serialised with it in _meta)
        hopts = self._meta.get(_HANDLE_OPTS)
        if hopts:
            o.update(hopts)
        if "enable_task_events" in opts:
            o["enable_task_events"] = opts["enable_task_events"]
        refs = cw.submit_actor_task(self._actor_id, name, args, kwargs, o)
        if nret == "streaming":
            return refs
        if nret == 1:
            return refs[0]
        if nret == 0:
            return None
        return refs

    def __repr__(self):
        return f"Actor({self._class_name}, {self._actor_id.hex()})"

    def __hash__(self):
        return hash(self._actor_id)

    def __eq__(self, other):
        return isinstance(other, ActorHandle) and other._actor_id == self._actor_id

    def __reduce__(self):
        cw = self._cw
        if cw is not None:
            cw.actor_escaped.add(self._actor_id)
        return (_rebuild_handle, (self._actor_id, self._class_name, self._meta, self._owner))

    def __del__(self):
        cw = self._cw
        if cw is not None:
            try:
                cw.actor_handle_deleted(self._actor_id, self._owner)
            except Exception:
                pass


def _rebuild_handle(actor_id, class_name, meta, owner):
    h = ActorHandle(actor_id, class_name, meta, owner)
    if h._cw is not None:
        h._cw._subscribe_actor(actor_id)
    return h


class ActorClass:
    def __init__(self, cls, options):
        _opt.validate(options, actor=True)
        self._cls = cls
        self._default_options = options
        self._keys = {}
        self._meta = _method_meta(cls)
        self.__name__ = cls.__name__
        self.__qualname__ = getattr(cls, "__qualname__", cls.__name__)
        self.__doc__ = cls.__doc__
        self.__module__ = cls.__module__

    def __call__(self, *args, **kwargs):
        raise TypeError(f"Actors cannot be instantiated directly. Instead of "
                        f"'{self._cls.__name__}()', use '{self._cls.__name__}.remote()'.")

    def remote(self, *args, **kwargs):
        return self._remote(args, kwargs, self._default_options)

    def options(self, **options):
        _opt.validate(options, actor=True)
        merged = dict(self._default_options)
        merged.update(options)
        parent = self

        class _Opt:
            def remote(self, *args, **kwargs):
                return parent._remote(args, kwargs, merged)

            def bind(self, *args, **kwargs):
                from ray_amd.dag import ClassNode

                return ClassNode(parent, args, kwargs, merged)

        return _Opt()

    def bind(self, *args, **kwargs):
        from ray_amd.dag import ClassNode

        return ClassNode(self, args, kwargs, self._default_options)

    def _remote(self, args, kwargs, opts):
        from ray_amd._private import worker as W
        from ray_amd._private.ids import random_bytes

        cw = W._check_connected()
        key = self._keys.get(_cw_key(cw))
        if key is None:
            key = cw.export(self._cls)
            self._keys[_cw_key(cw)] = key
        max_conc = opts.get("max_concurrency")
        if max_conc is None:
            max_conc = 1000 if self._meta.get("__is_async__") else 1
        groups = opts.get("concurrency_groups") or getattr(self._cls,
                                                           "__ray_amd_concurrency_groups__", None)
        o = {
            "resources": _opt.resources_of(opts, actor=True),
            "strategy": _opt.strategy_of(opts),
            "name": opts.get("name"), "namespace": opts.get("namespace"),
            "lifetime": opts.get("lifetime") or _default_lifetime(),
            "max_restarts": opts.get("max_restarts", 0),
            "max_task_retries": opts.get("max_task_retries", 0),
            "max_concurrency": max_conc, "concurrency_groups": groups,
            "runtime_env": opts.get("runtime_env"), "get_if_exists": opts.get("get_if_exists"),
        }
        aid = random_bytes(16)
        res = cw.create_actor(aid, key, args, kwargs, o, self._cls.__name__, self._meta)
        if res and res.get("existing"):
            h = ActorHandle(res["existing"], res["class_name"], res["method_meta"], res["owner"])
            cw._subscribe_actor(res["existing"])
            return h
        if o["name"] or o["lifetime"] == "detached":
            cw.actor_escaped.add(aid)
        meta = self._meta
        hopts = {k: opts[k] for k in ("max_pending_calls", "enable_task_events")
                 if opts.get(k) is not None and (k != "max_pending_calls" or opts[k] != -1)}
        if hopts:
            meta = dict(meta, **{_HANDLE_OPTS: hopts})
        return ActorHandle(aid, self._cls.__name__, meta, cw.addr)


def _default_lifetime():
    """JobConfig(default_actor_lifetime="detached") applies to actors created by the driver
    (reference: job_config.py set_default_actor_lifetime)."""
    from ray_amd._private import worker as W

    jc = getattr(W.global_worker, "job_config", None)
    if jc is not None and jc.default_actor_lifetime == "detached":
        return "detached"
    return None


def exit_actor():
    """Terminate the current actor gracefully (reference: ray.actor.exit_actor)."""
    from ray_amd._private import worker as W
    from ray_amd._private.core_worker import _ActorExit

    cw = W.global_worker.core
    if cw is None or cw.actor_id is None:
        raise TypeError("exit_actor API is called on a non-actor worker.")
    raise _ActorExit()


def _reset():
    pass


weakref  # noqa: B018
