"""Ray Data tests (modelled on python/ray/data/tests/test_map.py, test_all_to_all.py,
test_consumption.py, test_parquet.py, test_streaming_integration.py, preprocessors)."""

import numpy as np
import pandas as pd
import pytest

import ray_amd as ray
import ray_amd.data as rd
from ray_amd.data import preprocessors as pp


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_range_map_filter(cluster):
    ds = rd.range(100, override_num_blocks=7)
    assert ds.count() == 100
    out = ds.map(lambda r: {"id": r["id"], "sq": r["id"] ** 2}).filter(lambda r: r["id"] % 2 == 0)
    rows = out.take_all()
    assert len(rows) == 50 and rows[3] == {"id": 6, "sq": 36}
    b = ds.map_batches(lambda b: {"id": b["id"] * 10}, batch_size=16).take_batch(5)
    assert list(b["id"]) == [0, 10, 20, 30, 40]
    assert ds.flat_map(lambda r: [r, r]).count() == 200
    assert ds.sum("id") == 4950 and ds.min("id") == 0 and ds.max("id") == 99
    assert abs(ds.mean("id") - 49.5) < 1e-9 and abs(ds.std("id") - np.std(np.arange(100),
                                                                         ddof=1)) < 1e-6


class AddConst:
    def __init__(self, c):
        self.c = c

    def __call__(self, b):
        return {"id": b["id"] + self.c}


def test_actor_pool_map(cluster):
    ds = rd.range(64, override_num_blocks=8).map_batches(AddConst, fn_constructor_args=(1000,),
                                                         concurrency=2, batch_size=8)
    assert sorted(r["id"] for r in ds.take_all()) == list(range(1000, 1064))


def test_all_to_all(cluster):
    ds = rd.range(200, override_num_blocks=5)
    s = ds.random_shuffle(seed=1)
    ids = [r["id"] for r in s.take_all()]
    assert sorted(ids) == list(range(200)) and ids != list(range(200))
    assert ds.repartition(3).num_blocks() == 3 and ds.repartition(3).count() == 200
    srt = s.sort("id", descending=True)
    assert [r["id"] for r in srt.take(5)] == [199, 198, 197, 196, 195]
    u = ds.union(rd.range(10))
    assert u.count() == 210
    z = rd.range(10).zip(rd.range(10).map(lambda r: {"x": r["id"] * 2}))
    assert z.take(2) == [{"id": 0, "x": 0}, {"id": 1, "x": 2}]
    parts = ds.split(3, equal=True)
    assert [p.count() for p in parts] == [66, 66, 66]
    a, b = ds.train_test_split(0.25)
    assert (a.count(), b.count()) == (150, 50)
    assert ds.limit(7).count() == 7


def test_groupby(cluster):
    items = [{"k": i % 3, "v": float(i)} for i in range(30)]
    ds = rd.from_items(items)
    c = {r["k"]: r["count()"] for r in ds.groupby("k").count().take_all()}
    assert c == {0: 10, 1: 10, 2: 10}
    s = {r["k"]: r["sum(v)"] for r in ds.groupby("k").sum("v").take_all()}
    assert s[0] == sum(range(0, 30, 3))
    m = ds.groupby("k").map_groups(lambda g: {"k": g["k"][:1], "n": np.array([len(g["v"])])})
    assert sorted((r["k"], r["n"]) for r in m.take_all()) == [(0, 10), (1, 10), (2, 10)]


def test_iter_batches_and_torch(cluster):
    import torch

    ds = rd.range_tensor(100, shape=(3, 2), override_num_blocks=4)
    sizes = [len(b["data"]) for b in ds.iter_batches(batch_size=32)]
    assert sizes == [32, 32, 32, 4]
    tb = list(ds.iter_torch_batches(batch_size=50, dtypes=torch.float32))
    assert tb[0]["data"].shape == (50, 3, 2) and tb[0]["data"].dtype == torch.float32
    shuffled = [int(b["data"][0, 0, 0]) for b in ds.iter_batches(batch_size=10,
                                                                  local_shuffle_buffer_size=50,
                                                                  local_shuffle_seed=0)]
    assert len(shuffled) == 10
    df = ds.limit(3).map_batches(lambda b: b, batch_format="pandas").to_pandas()
    assert len(df) == 3


def test_io_roundtrip(cluster, tmp_path):
    df = pd.DataFrame({"a": np.arange(20), "b": np.arange(20) * 0.5})
    ds = rd.from_pandas(df)
    ds.write_parquet(str(tmp_path / "pq"))
    back = rd.read_parquet(str(tmp_path / "pq"))
    assert back.count() == 20 and back.sum("a") == 190
    ds.write_csv(str(tmp_path / "csv"))
    assert rd.read_csv(str(tmp_path / "csv")).count() == 20
    ds.write_json(str(tmp_path / "js"))
    assert rd.read_json(str(tmp_path / "js")).sum("a") == 190
    (tmp_path / "t.txt").write_text("x\ny\n\nz\n")
    assert rd.read_text(str(tmp_path / "t.txt")).count() == 3
    np.save(tmp_path / "arr.npy", np.ones((5, 2)))
    assert rd.read_numpy(str(tmp_path / "arr.npy")).count() == 5
    assert str(rd.from_pandas(df).schema()).startswith("Column names")


def test_preprocessors(cluster):
    ds = rd.from_items([{"x": float(i), "c": "abc"[i % 3]} for i in range(10)])
    sc = pp.StandardScaler(["x"]).fit(ds)
    xs = np.array([r["x"] for r in sc.transform(ds).take_all()])
    assert abs(xs.mean()) < 1e-9 and abs(xs.std(ddof=1) - 1) < 1e-9
    mm = pp.MinMaxScaler(["x"]).fit_transform(ds)
    assert mm.max("x") == 1.0 and mm.min("x") == 0.0
    oh = pp.OneHotEncoder(["c"]).fit_transform(ds).take(1)[0]["c"]
    assert list(oh) == [1, 0, 0]
    ch = pp.Chain(pp.OrdinalEncoder(["c"]), pp.Concatenator(["x", "c"], "f")).fit_transform(ds)
    assert ch.take(2)[1]["f"].tolist() == [1.0, 1.0]


def test_streaming_split_for_train(cluster):
    ds = rd.range(100, override_num_blocks=10)
    its = ds.streaming_split(2, equal=True)

    @ray.remote
    def consume(it):
        return sum(len(b["id"]) for b in it.iter_batches(batch_size=7))

    counts = ray.get([consume.remote(i) for i in its])
    assert sum(counts) == 100 and min(counts) >= 40


def test_streaming_split_equal_exact_rows(cluster):
    """equal=True: identical row counts per consumer, remainder dropped (reference:
    OutputSplitter equal=True); every delivered row is distinct."""
    ds = rd.range(103, override_num_blocks=7)
    its = ds.streaming_split(3, equal=True)

    @ray.remote
    def consume(it):
        out = []
        for b in it.iter_batches(batch_size=10):
            out.extend(int(x) for x in b["id"])
        return out

    parts = ray.get([consume.remote(i) for i in its])
    assert [len(p) for p in parts] == [34, 34, 34]
    allrows = sum(parts, [])
    assert len(set(allrows)) == len(allrows)
