"""Task pipelining on saturated nodes (ray_amd/_private/core_worker.py PIPELINE_DEPTH): while
lease requests of a scheduling class go unanswered, the owner queues a second task on each
leased worker. The reference submits one task per lease (src/ray/core_worker/transport/
direct_task_transport.cc OnWorkerIdle); these tests pin that pipelining never changes what
a program observes:

* a task blocked in ``ray.get`` hands the tasks queued behind it back to their owner, so a
  task waiting for a LATER task of the same class still finishes;
* a task that busy-waits for a later task (no ray.get) gets it stolen back onto the next
  worker that goes idle;
* results, ordering-independent sums and retries are unchanged under saturation.
"""

import os
import time

import pytest

import ray_amd as ray


@pytest.fixture(scope="module")
def two_cpus():
    ray.init(num_cpus=2)
    yield
    ray.shutdown()


def test_many_small_tasks_under_saturation(two_cpus):
    @ray.remote
    def sq(i):
        return i * i

    from ray_amd._private.worker import global_worker

    for _ in range(3):
        refs = [sq.remote(i) for i in range(3000)]
        assert sum(ray.get(refs)) == sum(i * i for i in range(3000))
    assert global_worker.core.pipeline_stats["pipelined"] > 0  # the path under test ran


def test_blocked_task_returns_its_queue(two_cpus):
    """Each waiter ray.get()s the result of a task submitted AFTER it (handed over through
    an actor mailbox); on a saturated 2-CPU node that later task may be pipelined behind
    its own waiter, which must give it back when it blocks."""

    @ray.remote
    class Box:
        def __init__(self):
            self.v = None

        def put(self, v):
            self.v = v

        def get(self):
            return self.v

    @ray.remote
    def later(i):
        time.sleep(0.01)
        return i

    @ray.remote
    def waiter(box):
        t0 = time.time()
        while time.time() - t0 < 30:
            r = ray.get(box.get.remote())
            if r is not None:
                return ray.get(r[0]) + 1000
            time.sleep(0.005)
        return -1

    @ray.remote
    def filler():
        time.sleep(0.05)
        return 0

    fill = [filler.remote() for _ in range(20)]
    outs = []
    for i in range(6):
        b = Box.remote()
        outs.append(waiter.remote(b))
        b.put.remote([later.remote(i)])  # list-wrapped: the ref itself, not its value
    assert ray.get(outs, timeout=90) == [1000 + i for i in range(6)]
    ray.get(fill)


def test_busy_wait_dependency_is_stolen_back(two_cpus, tmp_path):
    """t1 polls for a file that t2 creates (no ray.get: nothing hands the queue back).
    With t2 pipelined behind t1, the idle worker must steal t2."""
    flag = str(tmp_path / "flag")

    @ray.remote
    def filler():
        time.sleep(0.2)
        return 0

    @ray.remote
    def poll_for(path):
        t0 = time.time()
        while not os.path.exists(path):
            if time.time() - t0 > 30:
                return "timeout"
            time.sleep(0.01)
        return "seen"

    @ray.remote
    def create(path):
        open(path, "w").close()
        return "made"

    fills = [filler.remote() for _ in range(6)]
    t1 = poll_for.remote(flag)
    t2 = create.remote(flag)
    assert ray.get([t1, t2], timeout=60) == ["seen", "made"]
    ray.get(fills)
    print(dict(global_worker_stats()))


def global_worker_stats():
    from ray_amd._private.worker import global_worker

    return global_worker.core.pipeline_stats


def test_pipelining_disabled_by_env_matches(monkeypatch):
    from ray_amd._private import core_worker as cwm

    assert cwm.PIPELINE_DEPTH >= 1
    assert cwm.CoreWorker._pipelinable({"nret": 1, "retries": 3})
    assert not cwm.CoreWorker._pipelinable({"nret": 1, "retries": 0})
    assert not cwm.CoreWorker._pipelinable({"nret": -1, "retries": 3})
    assert not cwm.CoreWorker._pipelinable({"nret": 1, "retries": 3, "max_calls": 1})


def test_fresh_lease_steals_pipelined_task(two_cpus):
    """Long tasks saturate the node, so later ones get pipelined behind them. Once a worker
    frees up (a short task ends), its idle lease takes back a queued long task instead of
    leaving it behind a running one: all long tasks finish in about two task-lengths, not
    three."""

    @ray.remote
    def long(t):
        time.sleep(t)
        return 1

    t0 = time.time()
    refs = [long.remote(1.5) for _ in range(4)]
    assert sum(ray.get(refs, timeout=60)) == 4
    assert time.time() - t0 < 4.4  # 2 CPUs: two rounds of 1.5 s (+ startup), never three
