"""Ray Data operator semantics against pandas / numpy references (modelled on
python/ray/data/tests/test_map.py, test_sort.py, test_groupby / test_all_to_all.py,
test_consumption.py, test_split.py, test_zip.py, test_union.py): every transform is run
over several blocks and compared with the same computation done eagerly."""

import numpy as np
import pandas as pd
import pytest

import ray_amd as ray
import ray_amd.data as rd


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _df(ds):
    return ds.to_pandas().reset_index(drop=True)


def _frame(n=97, seed=0):
    rng = np.random.default_rng(seed)
    return pd.DataFrame({"k": rng.integers(0, 7, n), "x": rng.normal(size=n),
                         "i": np.arange(n)})


def test_map_flat_map_filter_chain(cluster):
    ds = rd.range(50, override_num_blocks=7)
    out = (ds.map(lambda r: {"id": r["id"], "sq": r["id"] ** 2})
             .filter(lambda r: r["sq"] % 3 == 0)
             .flat_map(lambda r: [{"v": r["id"]}, {"v": -r["id"]}]))
    vals = sorted(r["v"] for r in out.take_all())
    want = sorted(v for i in range(50) if (i * i) % 3 == 0 for v in (i, -i))
    assert vals == want


@pytest.mark.parametrize("fmt", ["numpy", "pandas"])
def test_map_batches_formats_and_sizes(cluster, fmt):
    ds = rd.range(103, override_num_blocks=5)

    def f(b):
        if fmt == "pandas":
            assert isinstance(b, pd.DataFrame)
            b = b.assign(y=b["id"] * 2)
        else:
            assert isinstance(b["id"], np.ndarray)
            b = {"id": b["id"], "y": b["id"] * 2}
        return b

    out = _df(ds.map_batches(f, batch_format=fmt, batch_size=10))
    assert len(out) == 103
    assert (out.sort_values("id")["y"].to_numpy() == np.arange(103) * 2).all()


def test_add_drop_select_rename_columns(cluster):
    df = _frame()
    ds = rd.from_pandas(df).repartition(4)
    ds2 = ds.add_column("z", lambda b: b["x"] * 2)
    assert set(ds2.columns()) == {"k", "x", "i", "z"}
    got = _df(ds2.select_columns(["i", "z"])).sort_values("i")
    assert np.allclose(got["z"].to_numpy(), df["x"].to_numpy() * 2)
    assert set(ds2.drop_columns(["x"]).columns()) == {"k", "i", "z"}
    assert set(ds.rename_columns({"x": "value"}).columns()) == {"k", "value", "i"}


@pytest.mark.parametrize("descending", [False, True])
def test_sort_matches_pandas(cluster, descending):
    df = _frame(211, seed=3)
    ds = rd.from_pandas(df).repartition(6)
    got = _df(ds.sort("x", descending=descending))
    want = df.sort_values("x", ascending=not descending).reset_index(drop=True)
    assert np.allclose(got["x"].to_numpy(), want["x"].to_numpy())
    assert (got["i"].to_numpy() == want["i"].to_numpy()).all()


def test_groupby_aggregations_match_pandas(cluster):
    df = _frame(300, seed=5)
    ds = rd.from_pandas(df).repartition(5)
    g = ds.groupby("k")
    cnt = _df(g.count()).sort_values("k")
    want = df.groupby("k").size()
    assert (cnt.iloc[:, 1].to_numpy() == want.to_numpy()).all()
    for agg, pfn in (("sum", "sum"), ("mean", "mean"), ("min", "min"), ("max", "max")):
        got = _df(getattr(g, agg)("x")).sort_values("k")
        assert np.allclose(got.iloc[:, 1].to_numpy(), getattr(df.groupby("k")["x"], pfn)()
                           .to_numpy()), agg
    std = _df(g.std("x")).sort_values("k")
    assert np.allclose(std.iloc[:, 1].to_numpy(), df.groupby("k")["x"].std(ddof=1).to_numpy())


def test_map_groups(cluster):
    df = _frame(120, seed=7)
    ds = rd.from_pandas(df).repartition(3)
    out = _df(ds.groupby("k").map_groups(
        lambda g: pd.DataFrame({"k": [g["k"].iloc[0]], "n": [len(g)]}), batch_format="pandas"))
    out = out.sort_values("k")
    assert (out["n"].to_numpy() == df.groupby("k").size().to_numpy()).all()


def test_global_aggregates(cluster):
    df = _frame(500, seed=9)
    ds = rd.from_pandas(df).repartition(7)
    assert ds.count() == 500
    assert np.isclose(ds.sum("x"), df["x"].sum())
    assert np.isclose(ds.mean("x"), df["x"].mean())
    assert np.isclose(ds.min("x"), df["x"].min()) and np.isclose(ds.max("x"), df["x"].max())
    assert np.isclose(ds.std("x"), df["x"].std(ddof=1))
    assert sorted(ds.unique("k")) == sorted(df["k"].unique().tolist())


def test_union_zip_limit(cluster):
    a = rd.range(30, override_num_blocks=3)
    b = rd.range(20, override_num_blocks=2).map(lambda r: {"id": r["id"] + 100})
    u = sorted(r["id"] for r in a.union(b).take_all())
    assert u == list(range(30)) + list(range(100, 120))
    z = _df(rd.range(25, override_num_blocks=4).zip(
        rd.range(25, override_num_blocks=3).map(lambda r: {"w": r["id"] * 10})))
    assert (z["w"].to_numpy() == z["id"].to_numpy() * 10).all()
    assert rd.range(1000, override_num_blocks=10).limit(17).count() == 17


def test_random_shuffle_is_a_permutation_and_seeded(cluster):
    ds = rd.range(200, override_num_blocks=5)
    s1 = [r["id"] for r in ds.random_shuffle(seed=1).take_all()]
    s2 = [r["id"] for r in ds.random_shuffle(seed=1).take_all()]
    assert sorted(s1) == list(range(200))
    assert s1 == s2 and s1 != list(range(200))


def test_splits(cluster):
    ds = rd.range(100, override_num_blocks=6)
    parts = ds.split(3, equal=True)
    counts = [p.count() for p in parts]
    assert counts == [33, 33, 33]
    a, b, c = ds.split_at_indices([10, 45])
    assert [a.count(), b.count(), c.count()] == [10, 35, 55]
    assert [r["id"] for r in b.take_all()] == list(range(10, 45))
    tr, te = ds.train_test_split(test_size=0.25)
    assert tr.count() == 75 and te.count() == 25
    ps = ds.split_proportionately([0.2, 0.3])
    assert [p.count() for p in ps] == [20, 30, 50]


def test_iter_batches_crosses_blocks(cluster):
    ds = rd.range(95, override_num_blocks=7)
    sizes = [len(b["id"]) for b in ds.iter_batches(batch_size=20)]
    assert sizes == [20, 20, 20, 20, 15]
    sizes = [len(b["id"]) for b in ds.iter_batches(batch_size=20, drop_last=True)]
    assert sizes == [20, 20, 20, 20]
    seen = np.concatenate([b["id"] for b in ds.iter_batches(batch_size=13)])
    assert (seen == np.arange(95)).all()


def test_take_batch_schema_show(cluster, capsys):
    ds = rd.from_items([{"a": i, "b": str(i)} for i in range(10)])
    tb = ds.take_batch(4)
    assert list(tb["a"]) == [0, 1, 2, 3]
    assert set(ds.schema().names if hasattr(ds.schema(), "names") else ds.columns()) == {"a", "b"}
    ds.show(2)
    assert "0" in capsys.readouterr().out


def test_parquet_and_csv_roundtrip(cluster, tmp_path):
    df = _frame(64, seed=11)
    ds = rd.from_pandas(df).repartition(3)
    ds.write_parquet(str(tmp_path / "pq"))
    back = _df(rd.read_parquet(str(tmp_path / "pq"))).sort_values("i").reset_index(drop=True)
    assert np.allclose(back["x"].to_numpy(), df["x"].to_numpy())
    ds.write_csv(str(tmp_path / "csv"))
    back = _df(rd.read_csv(str(tmp_path / "csv"))).sort_values("i").reset_index(drop=True)
    assert (back["k"].to_numpy() == df["k"].to_numpy()).all()


def test_materialize_reuses_blocks(cluster):
    calls = []

    def f(b):
        calls.append(1)
        return b

    ds = rd.range(40, override_num_blocks=4).map_batches(f).materialize()
    n1 = ds.count()
    n2 = len(ds.take_all())
    assert n1 == n2 == 40
    assert ds.num_blocks() == 4


def test_lineage_serialization_copy_and_context(tmp_path):
    """reference: dataset.py:231 copy, :4634 has_serializable_lineage, :4654
    serialize_lineage, :4745 deserialize_lineage, :4786 context."""
    import ray_amd.data as rd

    ray.init(num_cpus=2, ignore_reinit_error=True)
    try:
        for i in range(3):
            rd.from_items([{"x": i * 10 + j} for j in range(10)]).write_parquet(
                str(tmp_path / f"p{i}"))
        ds = rd.read_parquet([str(tmp_path / f"p{i}") for i in range(3)]).map(
            lambda r: {"x": r["x"] * 2})
        assert ds.has_serializable_lineage()
        assert not rd.from_items([{"x": 1}]).has_serializable_lineage()
        with pytest.raises(ValueError):
            rd.from_items([{"x": 1}]).serialize_lineage()
        blob = ds.serialize_lineage()
        ds2 = rd.Dataset.deserialize_lineage(blob)
        assert sorted(r["x"] for r in ds2.take_all()) == sorted(2 * v for v in range(30))
        ctx = rd.DataContext.get_current()
        old = ctx.target_max_block_size
        try:
            ctx.target_max_block_size = 12345
            ds3 = rd.range(5)
        finally:
            ctx.target_max_block_size = old
        assert ds3.context.target_max_block_size == 12345  # a snapshot at creation
        c = rd.Dataset.copy(ds3)
        assert c is not ds3 and c.take_all() == ds3.take_all()
        d = rd.Dataset.copy(ds3, _deep_copy=True)
        assert d._plan is not ds3._plan and d.count() == 5
    finally:
        ray.shutdown()
