"""Dask-on-Ray scheduler (reference: python/ray/util/dask/scheduler.py ray_dask_get).

``ray_dask_get(dsk, keys)`` runs a Dask task graph on the cluster: every graph entry that
computes something becomes one Ray task whose arguments are the ObjectRefs of the entries
it reads, so the object store carries intermediate results between workers and nothing
returns to the driver until the requested keys are fetched. Entries that are plain
literals are put into the store once; key aliases share their target's ref. Submission is
non-blocking, so the whole graph is in the scheduler before the first result is awaited.

It needs no dask: a graph is the classic dict spec (``util/dask/common.py``). With dask
installed it is also a ``dask.compute(..., scheduler=ray_dask_get)`` scheduler and
``enable_dask_on_ray()`` makes it the default."""

from __future__ import annotations

from typing import Any, Dict, Hashable

from ray_amd.util.dask.callbacks import active_callbacks, unpack_ray_callbacks
from ray_amd.util.dask.common import (deps_of, evaluate, flatten_keys, iskey, istask, pack,
                                      toposort)

_remote_exec = None


def _exec_fn(key, comp, dep_keys, pretask, posttask, *dep_values):
    """Body of one graph entry's Ray task (dependency refs arrive resolved)."""
    pre = [cb(key, list(dep_values)) for cb in pretask]
    result = evaluate(comp, dict(zip(dep_keys, dep_values)))
    for cb, st in zip(posttask, pre + [None] * (len(posttask) - len(pre))):
        cb(key, result, st)
    return result


def _remote():
    global _remote_exec
    if _remote_exec is None:
        import ray_amd as ray

        _remote_exec = ray.remote(_exec_fn)
    return _remote_exec


def _needs_task(comp, dsk) -> bool:
    if istask(comp):
        return True
    if isinstance(comp, list):
        return any(_needs_task(c, dsk) or iskey(c, dsk) for c in comp)
    return False


def ray_dask_get(dsk, keys, ray_callbacks=None, ray_persist=False, **kwargs):
    """Compute ``keys`` (a key or nested lists of keys) of graph ``dsk`` with Ray tasks.

    ``ray_persist=True`` returns ObjectRefs instead of values. ``num_workers`` / ``pool``
    (the reference's submission thread pool) are accepted and unused: submission here does
    not block. ``ray_remote_args`` (dict) become the tasks' ``.options``."""
    import ray_amd as ray

    kwargs.pop("num_workers", None)
    kwargs.pop("pool", None)
    remote_args = kwargs.pop("ray_remote_args", None) or {}
    dsk = dict(getattr(dsk, "dask", dsk))
    cbs = unpack_ray_callbacks(ray_callbacks if ray_callbacks is not None
                               else active_callbacks())
    leaves = list(flatten_keys(keys))
    refs: Dict[Hashable, Any] = {}
    fn = _remote()
    if remote_args:
        fn = fn.options(**remote_args)
    for key in toposort(dsk, leaves):
        comp = dsk[key]
        if iskey(comp, dsk) and not istask(comp):  # an alias of another entry
            refs[key] = refs[comp]
            continue
        dep_keys = list(deps_of(comp, dsk))
        if not _needs_task(comp, dsk):
            refs[key] = ray.put(comp)
            continue
        deps = {k: refs[k] for k in dep_keys}
        pre = None
        for cb in cbs.ray_presubmit:
            pre = cb(comp, key, deps)
            if pre is not None:
                break
        if pre is not None:
            refs[key] = ray.put(pre)
            continue
        ref = fn.options(name=f"dask:{key}").remote(key, comp, dep_keys, cbs.ray_pretask,
                                                     cbs.ray_posttask,
                                                     *[refs[k] for k in dep_keys])
        for cb in cbs.ray_postsubmit:
            cb(comp, key, deps, ref)
        refs[key] = ref
    out_refs = [refs[k] for k in leaves]
    for cb in cbs.ray_postsubmit_all:
        cb(out_refs, dsk)
    if ray_persist:
        result = pack(keys, {k: refs[k] for k in leaves})
    else:
        vals = ray.get(out_refs)
        result = pack(keys, dict(zip(leaves, vals)))
    for cb in cbs.ray_finish:
        cb(result)
    return result


def ray_dask_get_sync(dsk, keys, ray_callbacks=None, **kwargs):
    """The same graph evaluated in order in the calling process (debugging aid): the
    callbacks run as they would, with ``object_refs`` holding the dependency values."""
    dsk = dict(getattr(dsk, "dask", dsk))
    cbs = unpack_ray_callbacks(ray_callbacks if ray_callbacks is not None
                               else active_callbacks())
    leaves = list(flatten_keys(keys))
    values: Dict[Hashable, Any] = {}
    for key in toposort(dsk, leaves):
        comp = dsk[key]
        dep_keys = list(deps_of(comp, dsk))
        deps = {k: values[k] for k in dep_keys}
        pre = None
        for cb in cbs.ray_presubmit:
            pre = cb(comp, key, deps)
            if pre is not None:
                break
        if pre is not None:
            values[key] = pre
            continue
        values[key] = _exec_fn(key, comp, dep_keys, cbs.ray_pretask, cbs.ray_posttask,
                               *[values[k] for k in dep_keys])
        for cb in cbs.ray_postsubmit:
            cb(comp, key, deps, values[key])
    for cb in cbs.ray_postsubmit_all:
        cb([values[k] for k in leaves], dsk)
    result = pack(keys, values)
    for cb in cbs.ray_finish:
        cb(result)
    return result


def enable_dask_on_ray(shuffle="tasks", use_shuffle_optimization=True):
    """Make ``ray_dask_get`` dask's default scheduler (needs dask); returns the
    ``dask.config.set`` context so it can also be used in a ``with`` block."""
    try:
        import dask
    except ImportError as e:
        raise ImportError("enable_dask_on_ray needs the 'dask' package, which is not "
                          "installed; ray_dask_get(graph, keys) runs dict task graphs "
                          "without it") from e
    return dask.config.set(scheduler=ray_dask_get, shuffle=shuffle)


def disable_dask_on_ray():
    try:
        import dask
    except ImportError as e:
        raise ImportError("disable_dask_on_ray needs the 'dask' package") from e
    return dask.config.set(scheduler=None, shuffle=None)
