"""Dask-on-Ray scheduler callbacks (reference: python/ray/util/dask/callbacks.py).

A ``RayDaskCallback`` carries any of six hooks, given as constructor keywords or as
methods of a subclass:

* ``_ray_presubmit(task, key, deps)`` — driver, before a key's Ray task is submitted; a
  non-None return value becomes the key's result and no task is submitted;
* ``_ray_postsubmit(task, key, deps, object_ref)`` — driver, after submission;
* ``_ray_pretask(key, object_refs)`` — worker, before the key's computation runs; its
  return value is handed to ``_ray_posttask``;
* ``_ray_posttask(key, result, pre_state)`` — worker, after the computation;
* ``_ray_postsubmit_all(object_refs, dsk)`` — driver, once every task is submitted;
* ``_ray_finish(result)`` — driver, with the final result.

Callbacks are active inside ``with cb:`` (or ``cb.register()``), or are passed to one
``ray_dask_get(..., ray_callbacks=[...])`` call."""

from __future__ import annotations

import contextlib
import threading
from collections import namedtuple

CBS = ("ray_presubmit", "ray_postsubmit", "ray_pretask", "ray_posttask",
       "ray_postsubmit_all", "ray_finish")
CB_FIELDS = tuple(f"_{c}" for c in CBS)
RayCallback = namedtuple("RayCallback", CBS)
RayCallbacks = namedtuple("RayCallbacks", CBS)

_active: list = []
_lock = threading.Lock()


class RayDaskCallback:
    def __init__(self, **kwargs):
        for name in CB_FIELDS:
            fn = kwargs.pop(name, None) or kwargs.pop(name[1:], None)
            if fn is not None:
                setattr(self, name, fn)
        if kwargs:
            raise TypeError(f"unknown Dask-on-Ray callback(s): {sorted(kwargs)}")

    @property
    def _ray_callback(self) -> RayCallback:
        return RayCallback(*(getattr(self, f, None) for f in CB_FIELDS))

    def __enter__(self):
        self.register()
        return self

    def __exit__(self, *args):
        self.unregister()

    def register(self):
        with _lock:
            _active.append(self._ray_callback)

    def unregister(self):
        with _lock:
            cb = self._ray_callback
            for i in range(len(_active) - 1, -1, -1):
                if _active[i] == cb:
                    del _active[i]
                    break


def normalize_ray_callback(cb) -> RayCallback:
    if isinstance(cb, RayCallback):
        return cb
    if isinstance(cb, RayDaskCallback):
        return cb._ray_callback
    if isinstance(cb, tuple) and len(cb) == len(CBS):
        return RayCallback(*cb)
    raise TypeError("callbacks must be RayDaskCallback objects or RayCallback tuples")


def unpack_ray_callbacks(cbs) -> RayCallbacks:
    """Per-hook lists of the non-None hooks of ``cbs``."""
    cbs = [normalize_ray_callback(c) for c in (cbs or [])]
    return RayCallbacks(*([getattr(c, name) for c in cbs if getattr(c, name) is not None]
                          for name in CBS))


@contextlib.contextmanager
def local_ray_callbacks(callbacks=None):
    """Use ``callbacks`` (else the globally active ones) for the calls in this block."""
    global _active
    with _lock:
        saved = list(_active)
        if callbacks is not None:
            _active[:] = [normalize_ray_callback(c) for c in callbacks]
    try:
        yield list(_active)
    finally:
        with _lock:
            _active[:] = saved


def active_callbacks() -> list:
    with _lock:
        return list(_active)


class ProgressBarCallback(RayDaskCallback):
    """Counts submitted and finished keys (finish times come from the workers through a
    collector actor); ``report()`` prints a one-line summary."""

    def __init__(self):
        import ray_amd as ray

        @ray.remote(num_cpus=0)
        class _Progress:
            def __init__(self):
                self.submitted, self.finished = 0, 0

            def submit(self):
                self.submitted += 1

            def finish(self):
                self.finished += 1

            def result(self):
                return self.submitted, self.finished

        self._actor = _Progress.remote()
        actor = self._actor

        def _ray_postsubmit(task, key, deps, object_ref):
            actor.submit.remote()

        def _ray_posttask(key, result, pre_state):
            actor.finish.remote()

        super().__init__(ray_postsubmit=_ray_postsubmit, ray_posttask=_ray_posttask)

    def result(self):
        import ray_amd as ray

        return ray.get(self._actor.result.remote())

    def report(self):
        s, f = self.result()
        print(f"[dask-on-ray] {f}/{s} tasks finished", flush=True)
