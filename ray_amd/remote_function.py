"""@remote functions (reference: python/ray/remote_function.py)."""

from __future__ import annotations

import functools
import inspect

from ray_amd._private import options as _opt


def _cw_key(cw):
    """Cache key of a connection: the worker id (client connections: the object)."""
    return getattr(cw, "worker_id", None) or id(cw)


class RemoteFunction:
    def __init__(self, function, options: dict):
        _opt.validate(options, actor=False)
        self._function = function
        self._default_options = options
        self._keys = {}
        functools.update_wrapper(self, function)
        self._is_generator = inspect.isgeneratorfunction(function) or \
            inspect.isasyncgenfunction(function)

    def __call__(self, *args, **kwargs):
        raise TypeError(f"Remote functions cannot be called directly. Instead of running "
                        f"'{self._function.__name__}()', try '{self._function.__name__}.remote()'.")

    def remote(self, *args, **kwargs):
        return self._remote(args, kwargs, self._default_options)

    def options(self, **options):
        _opt.validate(options, actor=False)
        merged = dict(self._default_options)
        merged.update(options)
        parent = self

        class _Opt:
            def remote(self, *args, **kwargs):
                return parent._remote(args, kwargs, merged)

            def bind(self, *args, **kwargs):
                from ray_amd.dag import FunctionNode

                return FunctionNode(parent, args, kwargs, merged)

        return _Opt()

    def bind(self, *args, **kwargs):
        from ray_amd.dag import FunctionNode

        return FunctionNode(self, args, kwargs, self._default_options)

    def _key(self, cw):
        k = self._keys.get(_cw_key(cw))
        if k is None:
            k = cw.export(self._function)
            self._keys[_cw_key(cw)] = k
        return k

    def _remote(self, args, kwargs, opts):
        from ray_amd._private import worker as W

        cw = W._check_connected()
        nret = opts.get("num_returns")
        if nret is None:
            nret = "streaming" if self._is_generator else 1
        o = {
            "num_returns": nret,
            "resources": _opt.resources_of(opts, actor=False),
            "strategy": _opt.strategy_of(opts),
            "max_retries": opts.get("max_retries", 3),
            "retry_exceptions": opts.get("retry_exceptions", False),
            "runtime_env": opts.get("runtime_env"),
            "max_calls": opts.get("max_calls") or 0,
            "enable_task_events": opts.get("enable_task_events", True),
            "_generator_backpressure_num_objects":
                opts.get("_generator_backpressure_num_objects") or 0,
        }
        name = opts.get("name") or getattr(self._function, "__qualname__", "task")
        refs = cw.submit_task(self._key(cw), args, kwargs, o, name)
        if nret == "streaming":
            return refs
        if nret in (1, "dynamic"):
            return refs[0]
        if nret == 0:
            return None
        return refs
