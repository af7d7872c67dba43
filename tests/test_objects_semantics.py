"""Object and reference semantics (modelled on python/ray/tests/test_reference_counting.py,
test_reference_counting_2.py, test_object_spilling.py, test_streaming_generator.py,
test_get_or_put / test_basic_3.py): lifetimes, borrowing through containers, spilling
under pressure, generators, serialization of exotic values."""

import gc
import time

import numpy as np
import pytest

import ray_amd as ray
from ray_amd._private import worker as W


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4, object_store_memory=256 << 20)
    yield
    ray.shutdown()


def _in_store(ref):
    return W.global_worker.core.store.contains(ref._id)


def _wait_until(pred, timeout=10):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if pred():
            return True
        time.sleep(0.05)
    return pred()


def test_put_object_freed_after_del(cluster):
    ref = ray.put(np.zeros(4 << 20, np.uint8))
    assert _in_store(ref)
    oid = ref._id
    del ref
    gc.collect()
    assert _wait_until(lambda: not W.global_worker.core.store.contains(oid))


def test_ref_inside_list_keeps_object_alive(cluster):
    inner = ray.put(np.arange(1 << 20))
    outer = ray.put([inner])
    oid = inner._id
    del inner
    gc.collect()
    time.sleep(0.3)
    assert W.global_worker.core.store.contains(oid)  # held by the containing object
    got = ray.get(ray.get(outer)[0])
    assert got[-1] == (1 << 20) - 1
    del outer, got
    gc.collect()
    assert _wait_until(lambda: not W.global_worker.core.store.contains(oid))


def test_task_returning_a_ref_it_created(cluster):
    @ray.remote
    def make():
        return [ray.put(np.full(1 << 18, 7, np.int32))]

    (inner,) = ray.get(make.remote())
    assert int(ray.get(inner)[0]) == 7


def test_borrower_chain_through_actors(cluster):
    @ray.remote
    class Holder:
        def __init__(self):
            self.refs = []

        def keep(self, refs):
            self.refs.extend(refs)
            return len(self.refs)

        def read(self):
            return float(sum(ray.get(r).sum() for r in self.refs))

    h = Holder.remote()
    r = ray.put(np.ones(1 << 18))
    ray.get(h.keep.remote([r]))
    del r
    gc.collect()
    time.sleep(0.3)
    assert ray.get(h.read.remote()) == float(1 << 18)


def test_spilling_and_restore_under_pressure(cluster):
    # 24 x 16 MiB = 384 MiB through a 256 MiB store: the early objects spill
    refs = [ray.put(np.full(16 << 20, i % 251, np.uint8)) for i in range(24)]
    st = W.global_worker.core.store.stats()
    assert st["spilled_bytes"] > 0
    for i in (0, 1, 23):
        v = ray.get(refs[i])
        assert v[0] == i % 251 and v[-1] == i % 251
    del refs


def test_streaming_generator_backpressure_and_early_stop(cluster):
    @ray.remote
    def gen(n):
        for i in range(n):
            yield np.full(1000, i)

    g = gen.options(num_returns="streaming").remote(50)
    first = []
    for ref in g:
        first.append(int(ray.get(ref)[0]))
        if len(first) == 5:
            break
    assert first == [0, 1, 2, 3, 4]


def test_generator_error_surfaces_after_items(cluster):
    @ray.remote
    def gen():
        yield 1
        yield 2
        raise RuntimeError("gen failed")

    g = gen.options(num_returns="streaming").remote()
    vals = []
    with pytest.raises(Exception) as ei:
        for ref in g:
            vals.append(ray.get(ref))
    assert vals == [1, 2] and "gen failed" in str(ei.value)


def test_serialize_exotic_values(cluster):
    import collections
    import dataclasses
    import enum

    class Color(enum.Enum):
        RED = 1

    @dataclasses.dataclass
    class P:
        x: int
        y: list

    vals = [Color.RED, P(1, [2, 3]), collections.OrderedDict(a=1), {1, 2}, frozenset({3}),
            b"\x00bytes", bytearray(b"xy"), np.float16(1.5), np.array(["a", "bc"]),
            np.zeros((3, 4), order="F"), complex(1, 2), None, (1, (2, (3,)))]
    for v in vals:
        got = ray.get(ray.put(v))
        if isinstance(v, np.ndarray):
            assert np.array_equal(got, v) and got.dtype == v.dtype
        else:
            assert got == v, v

    @ray.remote
    def echo(x):
        return x

    assert ray.get(echo.remote(P(5, [6]))) == P(5, [6])
    f = ray.get(echo.remote(lambda z: z + 1))
    assert f(1) == 2


def test_get_list_preserves_order_and_duplicates(cluster):
    a, b = ray.put(1), ray.put(2)
    assert ray.get([a, b, a, b, b]) == [1, 2, 1, 2, 2]


def test_object_ref_hash_eq_and_pickle(cluster):
    import pickle

    r = ray.put(3)
    r2 = pickle.loads(pickle.dumps(r))
    assert r == r2 and hash(r) == hash(r2) and {r: 1}[r2] == 1
    assert ray.get(r2) == 3
