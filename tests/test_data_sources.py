"""Custom Datasource/Datasink, SQL, webdataset, images, random access, block order
(modelled on python/ray/data/tests/test_sql.py, test_webdataset.py, test_image.py,
test_random_access.py, test_datasink.py)."""

import os
import sqlite3

import numpy as np
import pytest

import ray_amd as ray
import ray_amd.data as rd


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_sql_roundtrip(cluster, tmp_path):
    db = str(tmp_path / "t.db")
    con = sqlite3.connect(db)
    con.execute("CREATE TABLE movie(title TEXT, year INT, score REAL)")
    con.executemany("INSERT INTO movie VALUES (?, ?, ?)",
                    [(f"m{i}", 1990 + i, i / 10) for i in range(25)])
    con.commit()
    con.close()
    factory = lambda: sqlite3.connect(db)  # noqa: E731
    ds = rd.read_sql("SELECT * FROM movie WHERE year >= 1995", factory, parallelism=4)
    rows = sorted(ds.take_all(), key=lambda r: r["year"])
    assert len(rows) == 20 and rows[0]["title"] == "m5" and rows[-1]["year"] == 2014
    assert ds.num_blocks() > 1  # sharded read
    c2 = sqlite3.connect(db)
    c2.execute("CREATE TABLE out(title TEXT, year INT, score REAL)")
    c2.commit()
    c2.close()
    n = ds.write_sql("INSERT INTO out VALUES (?, ?, ?)", factory)
    assert n == 20
    assert sqlite3.connect(db).execute("SELECT COUNT(*), SUM(year) FROM out").fetchone() == \
        (20, sum(range(1995, 2015)))


def test_webdataset_roundtrip(cluster, tmp_path):
    imgs = np.random.default_rng(0).integers(0, 255, (6, 8, 8, 3), dtype=np.uint8)
    rows = [{"__key__": f"s{i}", "png": imgs[i], "cls": i % 3, "txt": f"caption {i}",
             "json": {"i": i}} for i in range(6)]
    rd.from_items(rows).repartition(2).write_webdataset(str(tmp_path / "wds"))
    assert len(os.listdir(tmp_path / "wds")) == 2
    back = sorted(rd.read_webdataset(str(tmp_path / "wds")).take_all(),
                  key=lambda r: r["__key__"])
    assert [r["__key__"] for r in back] == [f"s{i}" for i in range(6)]
    assert back[2]["cls"] == 2 and back[4]["txt"] == "caption 4" and back[1]["json"] == {"i": 1}
    assert np.array_equal(np.asarray(back[3]["png"]), imgs[3])
    raw = rd.read_webdataset(str(tmp_path / "wds"), decoder=False, suffixes=["txt"]).take(1)
    assert set(raw[0]) == {"__key__", "txt"} and isinstance(raw[0]["txt"], bytes)


def test_write_images_and_read_back(cluster, tmp_path):
    imgs = np.random.default_rng(1).integers(0, 255, (4, 16, 16, 3), dtype=np.uint8)
    rd.from_numpy(imgs).write_images(str(tmp_path / "img"), column="data")
    files = sorted(os.listdir(tmp_path / "img"))
    assert len(files) == 4 and files[0].endswith(".png")
    back = rd.read_images(str(tmp_path / "img")).take_all()
    assert sorted(int(np.asarray(r["image"]).sum()) for r in back) == \
        sorted(int(x.sum()) for x in imgs)


class _CountingSource(rd.Datasource):
    def __init__(self, n, k):
        self.n, self.k = n, k

    def get_read_tasks(self, parallelism):
        per = self.n // self.k
        return [rd.ReadTask(lambda s=s: {"x": np.arange(s, s + per)}, {"num_rows": per})
                for s in range(0, self.n, per)]


class _SumSink(rd.Datasink):
    def __init__(self):
        self.started = False

    def on_write_start(self):
        self.started = True

    def write(self, blocks, ctx):
        return int(sum(b["x"].sum() for b in blocks))

    def on_write_complete(self, results):
        return sum(results)


def test_custom_datasource_and_datasink(cluster):
    ds = rd.read_datasource(_CountingSource(100, 4))
    assert ds.count() == 100
    assert ds.map_batches(lambda b: {"x": b["x"] * 2}).write_datasink(_SumSink()) == 2 * 4950


def test_random_access_and_block_order(cluster):
    ds = rd.from_items([{"k": i * 3, "v": f"val{i}"} for i in range(200)]).repartition(5)
    ra = ds.to_random_access_dataset("k", num_workers=3)
    assert ray.get(ra.get_async(30)) == {"k": 30, "v": "val10"}
    assert ray.get(ra.get_async(31)) is None
    got = ra.multiget([0, 597, 300, 7])
    assert got[0]["v"] == "val0" and got[1]["v"] == "val199" and got[2]["v"] == "val100"
    assert got[3] is None
    assert "3 workers" in ra.stats()
    shuffled = ds.randomize_block_order(seed=1)
    assert sorted(r["k"] for r in shuffled.take_all()) == [i * 3 for i in range(200)]
    assert len(ds.to_pandas_refs()) == 5


def test_partitioned_write_and_hive_read(tmp_path):
    """write_parquet/csv(partition_cols=...) -> col=value/ directories; reads add the
    partition columns back (reference: Partitioning("hive")) and partition_filter prunes."""
    import os

    rows = [{"year": 2020 + i % 2, "kind": "ab"[i % 3 == 0], "x": i} for i in range(12)]
    for fmt in ("parquet", "csv"):
        out = str(tmp_path / fmt)
        ds = rd.from_items(rows)
        getattr(ds, f"write_{fmt}")(out, partition_cols=["year", "kind"])
        dirs = sorted(os.listdir(out))
        assert dirs == ["year=2020", "year=2021"]
        assert sorted(os.listdir(os.path.join(out, "year=2020"))) == ["kind=a", "kind=b"]
        back = getattr(rd, f"read_{fmt}")(out).take_all()
        assert sorted(int(r["x"]) for r in back) == list(range(12))
        for r in back:
            assert int(r["year"]) == 2020 + int(r["x"]) % 2
            assert r["kind"] == "ab"[int(r["x"]) % 3 == 0]
        only = getattr(rd, f"read_{fmt}")(out, partition_filter=lambda p: p["year"] == "2021")
        assert sorted(int(r["x"]) for r in only.take_all()) == [1, 3, 5, 7, 9, 11]
        plain = getattr(rd, f"read_{fmt}")(out, partitioning=None).take_all()
        assert "year" not in plain[0] and "kind" not in plain[0]
