"""Data operator options honoured (reference: Dataset.map / flat_map / filter /
map_batches signatures): filter(expr=...) column expressions, fn_args / fn_kwargs on
row operators, ray_remote_args (runtime_env, max_retries, ...) passed to the tasks and
actors the executor launches, unknown remote args rejected, concurrency on row ops."""
import os

import pytest

import ray_amd as ray
import ray_amd.data as rd


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _ds():
    return rd.from_items([{"id": i, "label": "abc"[i % 3], "x": float(i) / 2} for i in range(30)])


def test_filter_expressions(cluster):
    ds = _ds()
    assert [r["id"] for r in ds.filter(expr="id >= 27").take_all()] == [27, 28, 29]
    got = ds.filter(expr="label in ['a', 'c'] and not (id % 2 == 0)").take_all()
    assert [r["id"] for r in got] == [i for i in range(30) if i % 3 in (0, 2) and i % 2]
    assert ds.filter(expr="3 < id <= 5").count() == 2
    assert ds.filter(expr="x * 2 - id == 0").count() == 30
    assert ds.filter(expr="label not in ['a']").count() == 20
    with pytest.raises(Exception):
        ds.filter(expr="__import__('os').getcwd()").count()
    with pytest.raises(ValueError):
        ds.filter(lambda r: True, expr="id > 1")


def test_row_ops_fn_args_and_remote_args(cluster):
    ds = _ds()
    assert [r["y"] for r in ds.map(lambda r, k, off=0: {"y": r["id"] * k + off},
                                   fn_args=(3,), fn_kwargs={"off": 1}).take(3)] == [1, 4, 7]
    assert ds.flat_map(lambda r, n: [r] * n, fn_args=(2,)).count() == 60
    assert ds.filter(lambda r, lo: r["id"] >= lo, fn_args=(25,)).count() == 5

    def env(batch):
        batch["v"] = [os.environ.get("DATA_OPT_TEST", "")] * len(batch["id"])
        return batch

    out = ds.map_batches(env, runtime_env={"env_vars": {"DATA_OPT_TEST": "yes"}},
                         max_retries=1).take(2)
    assert [r["v"] for r in out] == ["yes", "yes"]
    with pytest.raises(ValueError, match="unsupported ray_remote_args"):
        ds.map_batches(env, bogus_option=1)
    assert ds.map(lambda r: r, concurrency=2).count() == 30
