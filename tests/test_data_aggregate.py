"""ray.data.aggregate (modelled on python/ray/data/tests/test_all_to_all.py aggregate
cases): built-ins against pandas/numpy, whole-dataset and grouped, null handling, a
user-defined AggregateFn (init / accumulate_row / merge / finalize)."""

import math

import numpy as np
import pandas as pd
import pytest

import ray_amd as ray
from ray_amd import data as rd
from ray_amd.data.aggregate import (AbsMax, AggregateFn, Count, Max, Mean, Min, Quantile,
                                    Std, Sum, Unique)


@pytest.fixture(scope="module", autouse=True)
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _df(n=200, seed=0):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({"g": rng.integers(0, 5, n), "x": rng.normal(size=n) * 10,
                         "y": rng.integers(-50, 50, n)})


def test_whole_dataset_builtins_match_pandas():
    df = _df()
    ds = rd.from_pandas(df).repartition(7)
    out = ds.aggregate(Count(), Sum("y"), Min("x"), Max("x"), Mean("x"), Std("x"),
                       Std("x", ddof=0, alias_name="std0"), AbsMax("y"),
                       Quantile("x", q=0.9), Unique("g"))
    assert out["count()"] == len(df)
    assert out["sum(y)"] == df.y.sum()
    assert out["min(x)"] == pytest.approx(df.x.min())
    assert out["max(x)"] == pytest.approx(df.x.max())
    assert out["mean(x)"] == pytest.approx(df.x.mean())
    assert out["std(x)"] == pytest.approx(df.x.std(ddof=1))
    assert out["std0"] == pytest.approx(df.x.std(ddof=0))
    assert out["abs_max(y)"] == df.y.abs().max()
    assert out["quantile(x)"] == pytest.approx(np.quantile(df.x, 0.9))
    assert out["unique(g)"] == set(df.g)


def test_grouped_builtins_match_pandas():
    df = _df(300, 1)
    ds = rd.from_pandas(df).repartition(5)
    rows = ds.groupby("g").aggregate(Count(), Mean("x"), Std("x"), Max("y"),
                                     Quantile("y", 0.5)).take_all()
    ref = df.groupby("g")
    assert [r["g"] for r in rows] == sorted(df.g.unique())
    for r in rows:
        sub = ref.get_group(r["g"])
        assert r["count()"] == len(sub)
        assert r["mean(x)"] == pytest.approx(sub.x.mean())
        assert r["std(x)"] == pytest.approx(sub.x.std(ddof=1))
        assert r["max(y)"] == sub.y.max()
        assert r["quantile(y)"] == pytest.approx(np.quantile(sub.y, 0.5))
    assert ds.groupby("g").std("x", ddof=0).take(1)[0]["std(x)"] == pytest.approx(
        ref.get_group(sorted(df.g.unique())[0]).x.std(ddof=0))


def test_nulls():
    ds = rd.from_items([{"v": 1.0}, {"v": float("nan")}, {"v": 3.0}])
    out = ds.aggregate(Sum("v"), Mean("v"), Count("v", ignore_nulls=True),
                       Sum("v", ignore_nulls=False, alias_name="strict"))
    assert out["sum(v)"] == 4.0 and out["mean(v)"] == 2.0
    assert out["count(v)"] == 2
    assert out["strict"] is None


def test_custom_aggregate_fn_rows_and_blocks():
    ds = rd.range(100).repartition(6)
    sum_sq = AggregateFn(init=lambda k: 0, accumulate_row=lambda a, r: a + r["id"] ** 2,
                         merge=lambda a, b: a + b, name="sum_sq")
    evens = AggregateFn(init=lambda k: 0,
                        accumulate_block=lambda a, b: a + int((b["id"] % 2 == 0).sum()),
                        merge=lambda a, b: a + b, finalize=lambda a: a * 10, name="evens10")
    out = ds.aggregate(sum_sq, evens)
    assert out == {"sum_sq": sum(i * i for i in range(100)), "evens10": 500}
    with pytest.raises(ValueError):
        AggregateFn(init=lambda k: 0, merge=lambda a, b: a)
    g = rd.from_items([{"k": i % 3, "v": i} for i in range(30)]).groupby("k").aggregate(
        AggregateFn(init=lambda k: [], accumulate_row=lambda a, r: a + [r["v"]],
                    merge=lambda a, b: a + b, finalize=lambda a: max(a) - min(a),
                    name="spread")).take_all()
    assert [r["spread"] for r in g] == [27, 27, 27]
    assert not math.isnan(rd.range(10).aggregate(Mean("id"))["mean(id)"])


def test_multi_key_sort_and_groupby_match_pandas():
    rng = np.random.default_rng(3)
    df = pd.DataFrame({"a": rng.integers(0, 3, 120), "b": rng.choice(["x", "y", "z"], 120),
                       "v": rng.normal(size=120)})
    ds = rd.from_pandas(df).repartition(6)
    got = ds.sort(["a", "b"], descending=[False, True]).to_pandas()
    exp = df.sort_values(["a", "b"], ascending=[True, False], kind="stable")
    assert list(zip(got.a, got.b)) == list(zip(exp.a, exp.b))
    got = ds.sort(["b", "a"]).to_pandas()
    exp = df.sort_values(["b", "a"], kind="stable")
    assert list(zip(got.b, got.a)) == list(zip(exp.b, exp.a))
    rows = ds.groupby(["a", "b"]).aggregate(Count(), Sum("v")).take_all()
    ref = df.groupby(["a", "b"])
    assert [(r["a"], r["b"]) for r in rows] == sorted(ref.groups.keys())
    for r in rows:
        sub = ref.get_group((r["a"], r["b"]))
        assert r["count()"] == len(sub) and r["sum(v)"] == pytest.approx(sub.v.sum())
    sizes = ds.groupby(["a", "b"]).map_groups(
        lambda g: {"a": g["a"][:1], "b": g["b"][:1], "n": np.array([len(g["v"])])}).take_all()
    assert sum(int(r["n"]) for r in sizes) == 120 and len(sizes) == len(ref.groups)


def test_dataset_convenience_aggregations():
    df = _df(150, 4)
    ds = rd.from_pandas(df).repartition(4)
    assert ds.sum("y") == df.y.sum()
    assert ds.std("x", ddof=0) == pytest.approx(df.x.std(ddof=0))
    assert ds.std("x") == pytest.approx(df.x.std(ddof=1))
    assert ds.mean(["x", "y"]) == pytest.approx([df.x.mean(), df.y.mean()])
    assert ds.min("y") == df.y.min() and ds.max("y") == df.y.max()


def test_empty_dataset_aggregates_to_null():
    ds = rd.range(10).filter(lambda r: r["id"] > 100)
    out = ds.aggregate(Count(), Sum("id"), Mean("id"), Max("id"))
    assert out == {"count()": 0, "sum(id)": None, "mean(id)": None, "max(id)": None}


def test_unique_keeps_values_with_nulls():
    """A None / NaN in the column adds one null entry instead of hiding every value."""
    ds = rd.from_items([{"a": 3}, {"a": None}, {"a": 1}, {"a": 3}]).repartition(2)
    assert ds.unique("a") == [1, 3, None]
    ds = rd.from_items([{"a": 1.5}, {"a": float("nan")}, {"a": -2.0}])
    assert ds.unique("a") == [-2.0, 1.5, None]
    assert rd.from_items([{"a": "y"}, {"a": "x"}]).unique("a") == ["x", "y"]


def test_groupby_equal_keys_across_dtypes_share_a_group():
    """int64 1 in one block and float64 1.0 / bool True in another hash to the same
    partition: groupby returns ONE group per equal key."""
    from ray_amd.data.dataset import _stable_hash

    assert _stable_hash(1) == _stable_hash(1.0) == _stable_hash(True) == _stable_hash(np.int8(1))
    assert _stable_hash(0.5) == _stable_hash(np.float32(0.5))
    a = rd.from_items([{"k": 1, "v": 1}, {"k": 2, "v": 1}])
    b = rd.from_items([{"k": 1.0, "v": 1}, {"k": 2.0, "v": 1}])
    out = a.union(b).groupby("k").count().take_all()
    assert len(out) == 2 and sorted(r["count()"] for r in out) == [2, 2]
