"""Dask-on-Ray scheduler on dict task graphs (reference: python/ray/util/dask/scheduler.py;
its tests use dask collections, which are not installed here — the graphs below are the
classic spec those collections lower to)."""
import operator

import pytest

import ray_amd as ray
from ray_amd.util.dask import (RayDaskCallback, local_ray_callbacks, ray_dask_get,
                               ray_dask_get_sync)
from ray_amd.util.dask.common import toposort


@pytest.fixture(scope="module")
def cluster():
    started = not ray.is_initialized()
    if started:
        ray.init(num_cpus=4)
    yield
    if started:
        ray.shutdown()


def _inc(x):
    return x + 1


def _graph():
    return {
        "a": 1,
        "b": (_inc, "a"),
        ("x", 0): (operator.mul, "b", 10),
        ("x", 1): (operator.add, ("x", 0), "a"),
        "c": [("x", 0), ("x", 1), (_inc, "b")],
        "d": (sum, "c"),
        "alias": "d",
        "lit": (1, 2),  # a tuple that is not a task is a literal
    }


def test_graph_results_and_nested_keys(cluster):
    dsk = _graph()
    assert ray_dask_get(dsk, "d") == 20 + 21 + 3
    assert ray_dask_get(dsk, [["alias", ("x", 1)], "lit"]) == [[44, 21], (1, 2)]
    assert ray_dask_get_sync(dsk, ["d", "c"]) == [44, [20, 21, 3]]


def test_persist_returns_refs(cluster):
    refs = ray_dask_get(_graph(), ["b", ("x", 0)], ray_persist=True)
    assert all(isinstance(r, ray.ObjectRef) for r in refs)
    assert ray.get(refs) == [2, 20]


def test_tasks_run_in_workers(cluster):
    import os

    pid = ray_dask_get({"p": (os.getpid,)}, "p")
    assert pid != os.getpid()


def test_callbacks_hooks(cluster):
    seen = {"post": [], "all": None, "finish": None}

    def presubmit(task, key, deps):
        if key == "b":
            return 100  # skip the task, use this value
        return None

    def postsubmit(task, key, deps, ref):
        seen["post"].append(key)

    def pretask(key, refs):
        return f"pre:{key}"

    def posttask(key, result, pre_state):
        assert pre_state == f"pre:{key}"

    cb = RayDaskCallback(ray_presubmit=presubmit, ray_postsubmit=postsubmit,
                         ray_pretask=pretask, ray_posttask=posttask,
                         ray_postsubmit_all=lambda refs, dsk: seen.__setitem__("all", len(refs)),
                         ray_finish=lambda r: seen.__setitem__("finish", r))
    with cb:
        out = ray_dask_get(_graph(), ("x", 1))
    assert out == 1001
    assert "b" not in seen["post"] and ("x", 0) in seen["post"]
    assert seen["all"] == 1 and seen["finish"] == 1001
    # not active outside the block; local_ray_callbacks scopes an explicit list
    assert ray_dask_get(_graph(), ("x", 1)) == 21
    with local_ray_callbacks([cb]):
        assert ray_dask_get(_graph(), ("x", 1)) == 1001


def test_cycle_is_an_error():
    with pytest.raises(RuntimeError, match="cycle"):
        toposort({"a": (_inc, "b"), "b": (_inc, "a")}, ["a"])


def test_task_error_propagates(cluster):
    def boom(x):
        raise ValueError("bad value")

    with pytest.raises(Exception, match="bad value"):
        ray_dask_get({"a": 1, "b": (boom, "a")}, "b")


def test_enable_needs_dask():
    from ray_amd.util.dask import enable_dask_on_ray

    try:
        import dask  # noqa: F401
        pytest.skip("dask installed")
    except ImportError:
        pass
    with pytest.raises(ImportError, match="dask"):
        enable_dask_on_ray()
