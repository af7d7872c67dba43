"""joblib backend, tqdm_ray, get_object_locations, remote pdb, annotations, log_once, _Timer
(modelled on python/ray/tests/test_joblib.py, test_tqdm_ray.py, test_object_locations
(test_get_locations), test_ray_debugger.py, util/tests/test_annotations.py)."""

import io
import os
import socket
import threading
import time
import warnings

import numpy as np
import pytest

import ray_amd as ray


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _sq(x):
    return x * x, os.getpid()


def test_joblib_backend_runs_batches_as_tasks(cluster):
    import joblib

    from ray_amd.util.joblib import register_ray

    register_ray()
    with joblib.parallel_backend("ray"):
        out = joblib.Parallel(n_jobs=-1)(joblib.delayed(_sq)(i) for i in range(100))
    assert [v for v, _ in out] == [i * i for i in range(100)]
    assert os.getpid() not in {p for _, p in out}  # ran in worker processes
    # explicit n_jobs and an exception propagates
    with joblib.parallel_backend("ray", n_jobs=2):
        assert joblib.Parallel()(joblib.delayed(abs)(-i) for i in range(5)) == [0, 1, 2, 3, 4]
        with pytest.raises(ZeroDivisionError):
            joblib.Parallel()(joblib.delayed(lambda v: 1 / v)(i) for i in range(3))


def test_get_object_locations(cluster):
    from ray_amd.experimental.locations import get_object_locations

    big = ray.put(np.zeros(1 << 20, dtype=np.uint8))
    small = ray.put(1)

    @ray.remote
    def make():
        return np.ones(1 << 20, dtype=np.uint8)

    made = make.remote()
    ray.get(made)
    locs = get_object_locations([big, small, made])
    node = ray.get_runtime_context().get_node_id()
    assert locs[big]["node_ids"] == [node] and locs[big]["object_size"] >= 1 << 20
    assert locs[made]["node_ids"] == [node]
    assert locs[small]["node_ids"] == []


def test_tqdm_ray_remote_bars_reach_driver(cluster):
    from ray_amd.experimental import tqdm_ray

    @ray.remote
    def work(n):
        bar = tqdm_ray.tqdm(total=n, desc="work", flush_interval_s=0.0)
        for _ in range(n):
            bar.update(1)
        bar.close()
        return n

    seen = []
    orig = tqdm_ray._manager.process
    tqdm_ray._manager.process = lambda st: seen.append(st) or orig(st)
    try:
        assert ray.get([work.remote(5), work.remote(7)]) == [5, 7]
        deadline = time.time() + 10
        while time.time() < deadline and sum(s["closed"] for s in seen) < 2:
            tqdm_ray.flush_driver_bars()
            time.sleep(0.1)
    finally:
        tqdm_ray._manager.process = orig
    done = [s for s in seen if s["closed"]]
    assert sorted(s["x"] for s in done) == [5, 7]
    assert all(s["desc"] == "work" for s in done)
    # driver-side bar draws directly and iterates
    assert list(tqdm_ray.tqdm(range(3), desc="local")) == [0, 1, 2]


def test_remote_pdb_breakpoint_and_client(cluster):
    from ray_amd.util import rpdb

    @ray.remote
    def buggy(x):
        y = x + 1
        rpdb.set_trace()
        return y * 2

    ref = buggy.remote(20)
    deadline = time.time() + 30
    bps = []
    while time.time() < deadline and not bps:
        bps = rpdb.list_breakpoints()
        time.sleep(0.2)
    assert bps, "breakpoint was not registered"
    b = bps[0]
    s = socket.create_connection((b["host"], b["port"]), timeout=20)
    f = s.makefile("rwb")

    def read_prompt():
        buf = b""
        while not buf.endswith(b"(ray-pdb) "):
            ch = f.read(1)
            assert ch, buf
            buf += ch
        return buf.decode()

    read_prompt()
    f.write(b"p y\n")
    f.flush()
    assert "21" in read_prompt()
    f.write(b"c\n")
    f.flush()
    assert ray.get(ref, timeout=30) == 42
    s.close()
    assert not rpdb.list_breakpoints()


def test_annotations_log_once_timer():
    from ray_amd.util.annotations import (Deprecated, DeveloperAPI, PublicAPI,
                                          RayDeprecationWarning, is_annotated)
    from ray_amd.util.debug import disable_log_once_globally, log_once, reset_log_once
    from ray_amd.util.timer import _Timer

    @PublicAPI
    def a():
        """Doc."""
        return 1

    @PublicAPI(stability="beta")
    class B:
        pass

    @DeveloperAPI
    def c():
        return 3

    @Deprecated(message="use a()")
    def d():
        return 4

    assert a() == 1 and c() == 3 and is_annotated(a) and is_annotated(B)
    assert "PublicAPI" in a.__doc__ and "beta" in B.__doc__
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        assert d() == 4
    assert any(issubclass(x.category, RayDeprecationWarning) for x in w)
    with pytest.raises(ValueError):
        PublicAPI(stability="bogus")(lambda: 0)

    assert log_once("k1") and not log_once("k1")
    reset_log_once("k1")
    assert log_once("k1")

    t = _Timer(window_size=3)
    for _ in range(5):
        with t:
            time.sleep(0.001)
        t.push_units_processed(10)
    assert t.count == 5 and t.mean > 0 and t.mean_units_processed == 10
    assert t.mean_throughput > 0
    disable_log_once_globally()
    assert not log_once("fresh")
    import ray_amd.util.debug as dbg

    dbg._disabled = False
