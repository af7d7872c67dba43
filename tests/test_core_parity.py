"""More core-semantics cases modelled on python/ray/tests/test_basic.py,
test_basic_2.py, test_actor.py, test_actor_failures.py and test_failure.py: each case is
the observable contract of the reference, re-checked under the round-5 task path
(saturation-gated pipelining, requeue on block, work stealing)."""

import asyncio
import os
import time

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.exceptions import GetTimeoutError, RayActorError, RayTaskError


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_get_list_raises_the_failing_tasks_error(cluster):
    @ray.remote
    def ok(i):
        return i

    @ray.remote
    def bad():
        raise KeyError("boom")

    refs = [ok.remote(1), bad.remote(), ok.remote(3)]
    with pytest.raises(RayTaskError) as ei:
        ray.get(refs)
    assert isinstance(ei.value, KeyError) or "KeyError" in str(ei.value)
    assert ray.get(refs[0]) == 1 and ray.get(refs[2]) == 3


def test_wait_argument_validation(cluster):
    r = ray.put(1)
    with pytest.raises(ValueError):
        ray.wait([r], num_returns=2)
    with pytest.raises((TypeError, ValueError)):
        ray.wait(r)  # not a list
    ready, rest = ray.wait([r], timeout=0)
    assert ready == [r] and rest == []


def test_get_timeout_zero_on_ready_and_pending(cluster):
    @ray.remote
    def slow():
        time.sleep(2)
        return 1

    assert ray.get(ray.put(5), timeout=0) == 5
    with pytest.raises(GetTimeoutError):
        ray.get(slow.remote(), timeout=0)


def test_actor_method_num_returns(cluster):
    @ray.remote
    class A:
        @ray.method(num_returns=2)
        def two(self):
            return 1, 2

        def three(self):
            return 1, 2, 3

    a = A.remote()
    x, y = a.two.remote()
    assert ray.get([x, y]) == [1, 2]
    r1, r2, r3 = a.three.options(num_returns=3).remote()
    assert ray.get([r1, r2, r3]) == [1, 2, 3]


def test_kill_with_restart_allowed_restarts_actor(cluster):
    @ray.remote(max_restarts=1)
    class C:
        def __init__(self):
            self.n = 0

        def inc(self):
            self.n += 1
            return self.n

        def pid(self):
            return os.getpid()

    c = C.remote()
    assert ray.get(c.inc.remote()) == 1
    p0 = ray.get(c.pid.remote())
    ray.kill(c, no_restart=False)
    deadline = time.time() + 30
    while True:
        try:
            p1 = ray.get(c.pid.remote(), timeout=10)
            break
        except RayActorError:
            assert time.time() < deadline
            time.sleep(0.2)
    assert p1 != p0
    assert ray.get(c.inc.remote()) == 1  # fresh state after the restart


def test_actor_created_inside_task_returned_handle(cluster):
    @ray.remote
    class Box:
        def __init__(self, v):
            self.v = v

        def get(self):
            return self.v

    @ray.remote
    def make():
        b = Box.options(lifetime="detached", name="made_in_task").remote(41)
        ray.get(b.get.remote())
        return b

    b = ray.get(make.remote())
    assert ray.get(b.get.remote()) == 41
    ray.kill(ray.get_actor("made_in_task"))


def test_worker_crash_without_retries_fails(cluster):
    from ray_amd.exceptions import WorkerCrashedError

    @ray.remote(max_retries=0)
    def die():
        os._exit(1)

    with pytest.raises((WorkerCrashedError, RayTaskError)):
        ray.get(die.remote(), timeout=60)


def test_force_cancel_kills_a_busy_worker(cluster):
    from ray_amd.exceptions import TaskCancelledError, WorkerCrashedError

    @ray.remote(max_retries=0)
    def spin():
        while True:
            pass

    r = spin.remote()
    time.sleep(0.5)
    ray.cancel(r, force=True)
    with pytest.raises((TaskCancelledError, WorkerCrashedError, RayTaskError)):
        ray.get(r, timeout=30)


def test_fractional_cpus_pack_two_per_cpu(cluster):
    """8 tasks of 0.5 CPU on 4 CPUs all run at once (max overlap of their run intervals is
    8; at 1 CPU each it would be 4)."""

    @ray.remote(num_cpus=0.5)
    def hold(t):
        t0 = time.time()
        time.sleep(t)
        return t0, time.time()

    spans = ray.get([hold.remote(3.0) for _ in range(8)], timeout=120)
    events = sorted([(a, 1) for a, _ in spans] + [(b, -1) for _, b in spans])
    cur = peak = 0
    for _, d in events:
        cur += d
        peak = max(peak, cur)
    assert peak == 8


def test_actor_init_error_surfaces_on_method_calls(cluster):
    @ray.remote
    class Broken:
        def __init__(self):
            raise ValueError("bad init")

        def f(self):
            return 1

    b = Broken.remote()
    with pytest.raises((RayActorError, RayTaskError)) as ei:
        ray.get(b.f.remote(), timeout=30)
    assert "bad init" in str(ei.value)


def test_ref_future_and_asyncio(cluster):
    @ray.remote
    def v(x):
        return x * 2

    assert v.remote(4).future().result(timeout=30) == 8

    async def main():
        return await v.remote(5)

    assert asyncio.run(main()) == 10


def test_large_argument_passed_by_value_is_put_once(cluster):
    @ray.remote
    def total(a):
        return float(a.sum())

    arr = np.ones(4 << 20, dtype=np.float32)  # 16 MB: above the inline limit
    assert ray.get([total.remote(arr) for _ in range(4)]) == [float(4 << 20)] * 4


def test_async_actor_max_concurrency_bound(cluster):
    @ray.remote(max_concurrency=3)
    class Gate:
        def __init__(self):
            self.now = 0
            self.peak = 0

        async def work(self):
            self.now += 1
            self.peak = max(self.peak, self.now)
            await asyncio.sleep(0.2)
            self.now -= 1

        async def peak_seen(self):
            return self.peak

    g = Gate.remote()
    ray.get([g.work.remote() for _ in range(9)])
    assert ray.get(g.peak_seen.remote()) == 3


def test_actor_ready_and_pool(cluster):
    from ray_amd.util import ActorPool

    @ray.remote
    class Sq:
        def f(self, x):
            return x * x

    actors = [Sq.remote() for _ in range(2)]
    ray.get([a.__ray_ready__.remote() for a in actors])
    pool = ActorPool(actors)
    assert sorted(pool.map_unordered(lambda a, v: a.f.remote(v), range(6))) == \
        [0, 1, 4, 9, 16, 25]


def test_many_dependent_tasks_complete_under_saturation(cluster):
    """A chain of tasks each waiting on its predecessor with ray.get inside, submitted
    faster than the node can run them (the pipelining requeue-on-block path)."""

    @ray.remote
    def step(prev_box, i):
        prev = ray.get(prev_box[0]) if prev_box else 0
        return prev + i

    refs = []
    for i in range(40):
        refs.append(step.remote([refs[-1]] if refs else [], i))
    assert ray.get(refs[-1], timeout=120) == sum(range(40))
