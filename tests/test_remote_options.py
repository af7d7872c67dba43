"""Remote options that change behaviour (reference: python/ray/_private/ray_option_utils.py):
enable_task_events=False keeps a task / actor out of the task-event stream (timeline),
max_pending_calls caps a handle's outstanding actor calls (PendingCallsLimitExceeded)."""
import time

import pytest

import ray_amd as ray
from ray_amd.exceptions import PendingCallsLimitExceeded


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


@ray.remote
def traced():
    return 1


@ray.remote
def untraced():
    return 2


def test_enable_task_events_false_keeps_task_out_of_timeline(cluster):
    assert ray.get(traced.remote()) == 1
    assert ray.get(untraced.options(enable_task_events=False).remote()) == 2

    @ray.remote(enable_task_events=False)
    class Quiet:
        def ping(self):
            return "q"

    q = Quiet.remote()
    assert ray.get(q.ping.remote()) == "q"
    time.sleep(1.5)  # workers flush task events about once a second
    names = {ev["name"] for ev in ray.timeline()}
    assert any("traced" in n for n in names)
    assert not any("untraced" in n for n in names)
    assert not any(n.endswith("ping") for n in names)


def test_max_pending_calls(cluster):
    @ray.remote(max_pending_calls=2)
    class Slow:
        def work(self, t):
            time.sleep(t)
            return t

    a = Slow.remote()
    ray.get(a.work.remote(0))
    r1, r2 = a.work.remote(0.5), a.work.remote(0.5)
    with pytest.raises(PendingCallsLimitExceeded):
        a.work.remote(0)
    assert ray.get([r1, r2]) == [0.5, 0.5]
    assert ray.get(a.work.remote(0)) == 0  # capacity is back once the calls finished


def test_generator_backpressure(cluster):
    """_generator_backpressure_num_objects=N: the generator runs at most N items ahead of
    what the caller has consumed."""
    @ray.remote
    class Progress:
        def __init__(self):
            self.n = 0

        def bump(self):
            self.n += 1

        def get(self):
            return self.n

    prog = Progress.remote()

    @ray.remote(num_returns="streaming")
    def gen(p, n):
        for i in range(n):
            ray.get(p.bump.remote())
            yield i

    g = gen.options(_generator_backpressure_num_objects=2).remote(prog, 20)
    first = ray.get(next(g))
    time.sleep(1.0)
    assert first == 0 and ray.get(prog.get.remote()) <= 3  # 1 consumed + 2 ahead
    assert [ray.get(r) for r in g] == list(range(1, 20))
    # without the option the generator runs to the end on its own
    prog2 = Progress.remote()
    g2 = gen.remote(prog2, 20)
    ray.get(next(g2))
    time.sleep(1.0)
    assert ray.get(prog2.get.remote()) == 20
