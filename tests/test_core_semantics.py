"""More core semantics (modelled on python/ray/tests/test_actor.py, test_actor_failures.py,
test_concurrency_group.py, test_basic_2.py, test_placement_group*.py, test_object_store /
test_get_or_put): ordering, concurrency, retries, options, placement strategies."""

import os
import threading
import time

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.exceptions import GetTimeoutError, RayActorError, RayTaskError
from ray_amd.util.placement_group import placement_group, remove_placement_group
from ray_amd.util.scheduling_strategies import PlacementGroupSchedulingStrategy


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4, resources={"special": 2})
    yield
    ray.shutdown()


@ray.remote
class Log:
    def __init__(self):
        self.items = []

    def add(self, x):
        self.items.append(x)
        return len(self.items)

    def get(self):
        return list(self.items)


def test_actor_calls_from_one_caller_execute_in_order(cluster):
    a = Log.remote()
    refs = [a.add.remote(i) for i in range(200)]
    assert ray.get(refs) == list(range(1, 201))
    assert ray.get(a.get.remote()) == list(range(200))


def test_actor_handle_passed_to_tasks(cluster):
    a = Log.remote()

    @ray.remote
    def push(h, base):
        return ray.get([h.add.remote(base + i) for i in range(5)])

    ray.get([push.remote(a, 100 * k) for k in range(4)])
    got = ray.get(a.get.remote())
    assert sorted(got) == sorted(100 * k + i for k in range(4) for i in range(5))
    for k in range(4):  # per-caller order preserved
        mine = [x for x in got if x // 100 == k]
        assert mine == sorted(mine)


def test_concurrency_groups_isolate_methods(cluster):
    @ray.remote(concurrency_groups={"io": 2, "compute": 1})
    class C:
        def __init__(self):
            self.ev = threading.Event()

        @ray.method(concurrency_group="io")
        def wait_io(self):
            return self.ev.wait(10)

        @ray.method(concurrency_group="io")
        def release(self):
            self.ev.set()
            return True

        @ray.method(concurrency_group="compute")
        def compute(self, x):
            return x * 2

    c = C.remote()
    w = c.wait_io.remote()
    # the compute group runs while an io method blocks, and a second io slot is free
    assert ray.get(c.compute.remote(21), timeout=10) == 42
    assert ray.get(c.release.remote(), timeout=10)
    assert ray.get(w, timeout=10)


def test_max_concurrency_threaded_actor_overlaps(cluster):
    @ray.remote(max_concurrency=4)
    class Sleeper:
        def nap(self):
            time.sleep(0.5)
            return threading.get_ident()

    s = Sleeper.remote()
    ray.get(s.nap.remote())
    t0 = time.time()
    idents = ray.get([s.nap.remote() for _ in range(4)])
    assert time.time() - t0 < 1.6
    assert len(set(idents)) > 1


def test_async_actor_interleaves(cluster):
    import asyncio

    @ray.remote
    class A:
        async def slow(self, x):
            await asyncio.sleep(0.3)
            return x

    a = A.remote()
    ray.get(a.slow.remote(0))
    t0 = time.time()
    assert ray.get([a.slow.remote(i) for i in range(10)]) == list(range(10))
    assert time.time() - t0 < 2.0


def test_max_task_retries_after_actor_restart(cluster, tmp_path):
    marker = tmp_path / "died"

    @ray.remote(max_restarts=1, max_task_retries=1)
    class Fragile:
        def maybe_die(self, path):
            if not os.path.exists(path):
                open(path, "w").close()
                os._exit(1)
            return "ok"

    f = Fragile.remote()
    assert ray.get(f.maybe_die.remote(str(marker)), timeout=60) == "ok"


def test_actor_dead_after_restarts_exhausted(cluster):
    @ray.remote(max_restarts=0)
    class Dies:
        def die(self):
            os._exit(1)

        def ping(self):
            return 1

    d = Dies.remote()
    assert ray.get(d.ping.remote()) == 1
    with pytest.raises(RayActorError):
        ray.get(d.die.remote(), timeout=30)
    with pytest.raises(RayActorError):
        ray.get(d.ping.remote(), timeout=30)


def test_get_if_exists_and_namespaces(cluster):
    a = Log.options(name="shared_log", get_if_exists=True).remote()
    b = Log.options(name="shared_log", get_if_exists=True).remote()
    ray.get(a.add.remote("x"))
    assert ray.get(b.get.remote()) == ["x"]
    assert ray.get(ray.get_actor("shared_log").get.remote()) == ["x"]
    with pytest.raises(ValueError):
        ray.get_actor("shared_log", namespace="some_other_ns")


def test_task_options_override_and_num_returns(cluster):
    @ray.remote(num_returns=2)
    def two(x):
        return x, x + 1

    a, b = two.remote(1)
    assert ray.get([a, b]) == [1, 2]

    @ray.remote
    def three(x):
        return x, x + 1, x + 2

    c, d, e = three.options(num_returns=3).remote(5)
    assert ray.get([c, d, e]) == [5, 6, 7]
    assert ray.get(three.remote(0)) == (0, 1, 2)  # options() left the function unchanged


def test_custom_resources_limit_concurrency(cluster):
    @ray.remote(resources={"special": 1}, num_cpus=0)
    def hold(t):
        time.sleep(t)
        return time.time()

    t0 = time.time()
    ends = ray.get([hold.remote(0.5) for _ in range(4)])
    # 2 units of "special": 4 tasks take two waves
    assert max(ends) - t0 >= 0.9


def test_placement_group_strategies(cluster):
    pg = placement_group([{"CPU": 1}, {"CPU": 1}], strategy="PACK")
    assert pg.wait(10)

    @ray.remote(num_cpus=1)
    def where():
        return ray.get_runtime_context().get_node_id()

    nodes = ray.get([where.options(scheduling_strategy=PlacementGroupSchedulingStrategy(
        pg, placement_group_bundle_index=i)).remote() for i in range(2)])
    assert len(nodes) == 2
    remove_placement_group(pg)
    pg2 = placement_group([{"CPU": 100}], strategy="STRICT_PACK")
    assert not pg2.wait(1)  # infeasible bundle: never ready
    remove_placement_group(pg2)


def test_put_get_numpy_readonly_and_large(cluster):
    x = np.arange(10_000_000, dtype=np.float32)
    ref = ray.put(x)
    y = ray.get(ref)
    assert np.array_equal(x, y)
    assert not y.flags.writeable  # zero-copy views of the store are immutable


def test_wait_fetch_local_and_timeout(cluster):
    @ray.remote
    def slow(t):
        time.sleep(t)
        return t

    refs = [slow.remote(0.05), slow.remote(5)]
    ready, pending = ray.wait(refs, num_returns=1, timeout=3, fetch_local=True)
    assert ready == [refs[0]] and pending == [refs[1]]
    with pytest.raises(GetTimeoutError):
        ray.get(refs[1], timeout=0.2)
    ray.cancel(refs[1], force=True)


def test_exception_chain_preserves_type(cluster):
    class MyErr(ValueError):
        pass

    @ray.remote
    def bad():
        raise MyErr("boom")

    with pytest.raises(MyErr):
        ray.get(bad.remote())
    try:
        ray.get(bad.remote())
    except RayTaskError as e:  # also a RayTaskError
        assert "boom" in str(e)
    except MyErr as e:
        assert isinstance(e, RayTaskError)


def test_nested_remote_calls_and_ray_get_inside_task(cluster):
    @ray.remote
    def leaf(x):
        return x + 1

    @ray.remote
    def mid(x):
        return sum(ray.get([leaf.remote(x + i) for i in range(3)]))

    @ray.remote
    def root():
        return ray.get([mid.remote(i) for i in range(4)])

    assert ray.get(root.remote()) == [sum(i + j + 1 for j in range(3)) for i in range(4)]
