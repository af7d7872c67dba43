"""The datasource package (reference: python/ray/data/datasource/): a custom
FileBasedDatasource through ``_read_stream``, partitioning styles and filters, metadata
providers, filename providers on writes, the format datasinks, the in-memory sources."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.csv as pc
import pytest

import ray_amd as ray
from ray_amd import data as rd
from ray_amd.data.datasource import (CSVDatasource, DummyOutputDatasink,
                                     FastFileMetadataProvider, FileBasedDatasource,
                                     FileExtensionFilter, FilenameProvider, Partitioning,
                                     PartitionStyle, PathPartitionFilter, PathPartitionParser,
                                     RandomIntRowDatasource, RangeDatasource, TorchDatasource,
                                     _CSVDatasink, _JSONDatasink, _NumpyDatasink,
                                     _ParquetDatasink)


@pytest.fixture(scope="module")
def cluster():
    started = not ray.is_initialized()
    if started:
        ray.init(num_cpus=4)
    yield
    if started:
        ray.shutdown()


class KVDatasource(FileBasedDatasource):
    """Lines 'k=v' -> rows (the reference's custom-datasource extension point)."""

    _FILE_EXTENSIONS = ["kv"]

    def _read_stream(self, f, path):
        keys, vals = [], []
        for line in f.read().decode().splitlines():
            k, v = line.split("=")
            keys.append(k)
            vals.append(int(v))
        yield pa.table({"k": keys, "v": vals})


def _tree(tmp_path):
    for yr in (2023, 2024):
        for mo in (1, 2):
            d = tmp_path / "t" / f"year={yr}" / f"month={mo}"
            d.mkdir(parents=True)
            (d / "a.kv").write_text(f"x={yr}\ny={mo}\n")
            (d / "ignore.txt").write_text("nope")
    (tmp_path / "t" / "_SUCCESS").write_text("")
    return str(tmp_path / "t")


def test_custom_file_datasource_with_hive_partitions(cluster, tmp_path):
    root = _tree(tmp_path)
    ds = rd.read_datasource(KVDatasource(root, include_paths=True))
    rows = sorted(ds.take_all(), key=lambda r: (r["year"], r["month"], r["k"]))
    assert len(rows) == 8 and len(ds.input_files()) == 4
    assert rows[0]["k"] == "x" and rows[0]["v"] == 2023 and rows[0]["year"] == "2023"
    assert rows[0]["path"].endswith("a.kv")


def test_partition_filter_and_typed_parser(cluster, tmp_path):
    root = _tree(tmp_path)
    flt = PathPartitionFilter.of(lambda p: p["year"] == "2024" and p["month"] == "2")
    ds = rd.read_datasource(KVDatasource(root, partition_filter=flt))
    assert sorted(r["v"] for r in ds.take_all()) == [2, 2024]
    part = Partitioning("hive", field_types={"year": int, "month": int})
    ds = rd.read_datasource(KVDatasource(root, partitioning=part))
    assert {r["year"] for r in ds.take_all()} == {2023, 2024}
    # a predicate over the values works as partition_filter too (ray_amd's older form)
    ds = rd.read_datasource(KVDatasource(root, partition_filter=lambda p: p["month"] == "1"))
    assert len(ds.take_all()) == 4


def test_directory_partitioning(cluster, tmp_path):
    for cc in ("us", "fr"):
        d = tmp_path / "d" / cc / "2020"
        d.mkdir(parents=True)
        (d / "f.csv").write_text("a\n1\n2\n")
    part = Partitioning(PartitionStyle.DIRECTORY, base_dir=str(tmp_path / "d"),
                        field_names=["country", "year"], field_types={"year": int})
    parser = PathPartitionParser(part)
    assert parser(str(tmp_path / "d" / "us" / "2020" / "f.csv")) == {"country": "us",
                                                                      "year": 2020}
    ds = rd.read_csv(str(tmp_path / "d"), partitioning=part)
    rows = ds.take_all()
    assert len(rows) == 4 and {r["country"] for r in rows} == {"us", "fr"}
    assert all(r["year"] == 2020 for r in rows)


def test_extension_filter_and_fast_meta_provider(cluster, tmp_path):
    root = _tree(tmp_path)
    f = FileExtensionFilter("kv")
    assert all(p.endswith(".kv") for p in f([os.path.join(root, "a.kv"),
                                             os.path.join(root, "b.txt")]))
    src = KVDatasource(root, meta_provider=FastFileMetadataProvider())
    assert src.estimate_inmemory_data_size() is None and len(src.input_files()) == 4
    assert KVDatasource(root).estimate_inmemory_data_size() > 0


class _Names(FilenameProvider):
    def get_filename_for_block(self, block, task_index, block_index):
        return f"custom_{task_index}_{block_index}.csv"


def test_filename_provider_and_format_datasinks(cluster, tmp_path):
    ds = rd.range(20, override_num_blocks=2).map(lambda r: {"id": r["id"],
                                                           "sq": r["id"] ** 2})
    out = tmp_path / "csv"
    n = ds.write_datasink(_CSVDatasink(str(out), filename_provider=_Names()))
    assert n == 20
    assert sorted(os.listdir(out)) == ["custom_0_0.csv", "custom_1_0.csv"]
    back = rd.read_datasource(CSVDatasource(str(out))).sort("id").take_all()
    assert [r["sq"] for r in back] == [i * i for i in range(20)]
    ds.write_datasink(_ParquetDatasink(str(tmp_path / "pq")))
    assert rd.read_parquet(str(tmp_path / "pq")).count() == 20
    ds.write_datasink(_JSONDatasink(str(tmp_path / "js")))
    assert rd.read_json(str(tmp_path / "js")).count() == 20
    ds.write_datasink(_NumpyDatasink(str(tmp_path / "np"), column="sq"))
    assert sorted(np.concatenate([np.atleast_1d(r["data"]) for r in
                                  rd.read_numpy(str(tmp_path / "np")).take_all()])) == \
        [i * i for i in range(20)]
    # Dataset.write_csv takes a FilenameProvider too
    ds.write_csv(str(tmp_path / "csv2"), filename_provider=_Names())
    assert sorted(os.listdir(tmp_path / "csv2")) == ["custom_0_0.csv", "custom_1_0.csv"]


def test_pyarrow_filesystem_reads(cluster, tmp_path):
    import pyarrow.fs as pafs

    (tmp_path / "x").mkdir()
    pc.write_csv(pa.table({"a": [1, 2, 3]}), str(tmp_path / "x" / "f.csv"))
    ds = rd.read_csv(str(tmp_path / "x"), filesystem=pafs.LocalFileSystem())
    assert ds.sum("a") == 6
    ds = rd.read_csv("file://" + str(tmp_path / "x"))
    assert ds.count() == 3


def test_in_memory_sources_and_dummy_sink(cluster):
    assert rd.read_datasource(RangeDatasource(10), parallelism=3).sum("id") == 45
    t = rd.read_datasource(RangeDatasource(4, block_format="tensor", tensor_shape=(2, 2)))
    assert t.take(1)[0]["data"].shape == (2, 2)
    r = rd.read_datasource(RandomIntRowDatasource(50, 3, seed=1), parallelism=2)
    assert r.count() == 50 and set(r.columns()) == {"c_0", "c_1", "c_2"}

    class Sq:
        def __len__(self):
            return 6

        def __getitem__(self, i):
            return i * i

    assert sorted(x["item"] for x in rd.read_datasource(TorchDatasource(Sq()),
                                                         parallelism=2).take_all()) == \
        [0, 1, 4, 9, 16, 25]
    sink = DummyOutputDatasink()
    assert rd.range(30).write_datasink(sink) == 30
