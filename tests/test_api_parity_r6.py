"""Round-6 API parity additions: experimental.load_package / set_resource /
get_object_locations, tune create_searcher / create_scheduler, data.NodeIdStr,
rllib.TFPolicy and util.ray_debugpy refusals (reference: python/ray/experimental/
__init__.py, tune/search/__init__.py, tune/schedulers/__init__.py)."""
import pytest

import ray_amd as ray


def test_load_package(tmp_path):
    (tmp_path / "interface.py").write_text(
        "import ray_amd as ray\n\n"
        "@ray.remote\n"
        "def add(a, b):\n    import os\n    return a + b, os.environ.get('PKG_FLAG')\n\n"
        "@ray.remote\n"
        "class Counter:\n    def __init__(self):\n        self.n = 0\n"
        "    def inc(self):\n        self.n += 1\n        return self.n\n")
    (tmp_path / "pkg.yaml").write_text(
        "name: demo\ndescription: a demo package\ninterface_file: interface.py\n"
        "runtime_env:\n  env_vars:\n    PKG_FLAG: 'on'\n")
    from ray_amd.experimental import load_package

    ray.init(num_cpus=2)
    try:
        pkg = load_package(str(tmp_path / "pkg.yaml"))
        assert pkg._runtime_env["working_dir"] == str(tmp_path)
        assert ray.get(pkg.add.remote(2, 3)) == (5, "on")
        c = pkg.Counter.remote()
        assert ray.get(c.inc.remote()) == 1
        from ray_amd.experimental import get_object_locations

        ref = ray.put(b"x" * (1 << 20))
        locs = get_object_locations([ref])
        assert locs[ref]["object_size"] >= 1 << 20
    finally:
        ray.shutdown()
    with pytest.raises(DeprecationWarning):
        from ray_amd.experimental import set_resource

        set_resource("foo", 1)


def test_tune_factories_and_refusals():
    from ray_amd.tune.schedulers import ASHAScheduler, FIFOScheduler, create_scheduler
    from ray_amd.tune.search import BasicVariantGenerator, create_searcher

    assert isinstance(create_scheduler("fifo"), FIFOScheduler)
    assert isinstance(create_scheduler("asha", metric="m", mode="max"), ASHAScheduler)
    assert isinstance(create_searcher("random"), BasicVariantGenerator)
    with pytest.raises(ValueError):
        create_scheduler("nope")
    import ray_amd.data as rd

    assert rd.NodeIdStr is str
    from ray_amd.rllib import TFPolicy

    with pytest.raises(ImportError, match="tensorflow"):
        TFPolicy(None, None, {})
    from ray_amd.util import ray_debugpy

    with pytest.raises(ImportError, match="debugpy"):
        ray_debugpy.set_trace()


def test_dummy_trainer_and_aliases():
    import ray_amd.data as rd
    from ray_amd.cloudpickle import dumps, loads
    from ray_amd.train import ScalingConfig
    from ray_amd.train.util import DummyTrainer
    from ray_amd.tune.analysis import ExperimentAnalysis  # noqa: F401
    from ray_amd.tune.experiment import Experiment, _convert_to_experiment_list

    assert loads(dumps(lambda x: x * 3))(2) == 6
    exps = _convert_to_experiment_list({"e1": {"run": lambda c: None}})
    assert len(exps) == 1 and isinstance(exps[0], Experiment)
    ray.init(num_cpus=4)
    try:
        r = DummyTrainer(scaling_config=ScalingConfig(num_workers=2),
                         datasets={"train": rd.range(4000)}, batch_size=500).fit()
        assert r.metrics["rows_read"] == 2000 and r.metrics["batches_read"] == 4
    finally:
        ray.shutdown()


def test_tune_utils():
    from ray_amd.tune.utils import (UtilMonitor, deep_update, diagnose_serialization,
                                    flatten_dict, merge_dicts, unflattened_lookup,
                                    warn_if_slow)

    assert flatten_dict({"a": {"b": 1, "c": {"d": 2}}, "e": 3}) == {"a/b": 1, "a/c/d": 2,
                                                                     "e": 3}
    assert merge_dicts({"a": {"b": 1}}, {"a": {"c": 2}}) == {"a": {"b": 1, "c": 2}}
    with pytest.raises(Exception):
        deep_update({"a": 1}, {"zz": 2})
    assert unflattened_lookup("a/1/b", {"a": [0, {"b": 7}]}) == 7
    assert unflattened_lookup("x/y", {}, default=None) is None
    import threading

    lock = threading.Lock()
    assert diagnose_serialization(lambda: 1) is True
    bad = diagnose_serialization(lambda: lock.acquire())
    assert "lock" in bad
    m = UtilMonitor(delay=0.05)
    import time

    time.sleep(0.2)
    m.stop()
    assert "cpu_util_percent" in m.get_data().get("perf", {})
    with warn_if_slow("noop"):
        pass


def test_workflow_filesystem_storage(tmp_path):
    import asyncio

    from ray_amd.workflow.storage import FilesystemStorage, KeyNotFoundError, Storage

    st = FilesystemStorage(str(tmp_path / "wf"))
    assert isinstance(st, Storage)

    async def run():
        k = st.make_key("wf1", "steps", "a")
        await st.put(k, {"x": 1}, is_json=True)
        await st.put(st.make_key("wf1", "steps", "b"), [1, 2, 3])
        assert await st.get(k, is_json=True) == {"x": 1}
        assert await st.scan_prefix("wf1/steps") == ["a", "b"]
        await st.delete_prefix("wf1")
        with pytest.raises(KeyNotFoundError):
            await st.get(k)

    asyncio.run(run())
    assert st.storage_url.startswith("file://")
