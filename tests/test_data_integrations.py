"""External-framework conversions of ray_amd.data (data/integrations.py): with the
framework missing they fail like the reference does — an ImportError naming the package —
and the legacy ``write_datasource`` path writes through a Datasink or a datasource's
``write(blocks)``."""
import pytest

import ray_amd as ray
import ray_amd.data as rd
from ray_amd.data import Datasink


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=2)
    yield
    ray.shutdown()


@pytest.mark.parametrize("fn,pkg", [("from_dask", "dask"), ("from_modin", "modin"),
                                    ("from_spark", "pyspark"), ("from_tf", "tensorflow"),
                                    ("from_mars", "pymars")])
def test_from_external_requires_package(fn, pkg):
    with pytest.raises(ImportError, match=pkg):
        getattr(rd, fn)(object())


def test_dataset_external_methods(cluster):
    ds = rd.range(10)
    for meth, args, pkg in (("to_dask", (), "dask"), ("to_tf", ("id", "id"), "tensorflow"),
                            ("to_modin", (), "modin"), ("to_spark", (None,), "pyspark")):
        with pytest.raises(ImportError, match=pkg):
            getattr(ds, meth)(*args)
    with pytest.raises(ImportError, match="tensorflow"):
        next(iter(ds.iter_tf_batches(batch_size=4)))


class _Collect(Datasink):
    def write(self, blocks, ctx):
        return sum(len(next(iter(b.values()))) if isinstance(b, dict) else b.num_rows
                   for b in blocks)

    def on_write_complete(self, results):
        return sum(results)


class _LegacySource:
    def __init__(self):
        self.rows = 0

    def write(self, blocks, **kw):
        self.rows = sum(b.num_rows for b in blocks)
        return self.rows


def test_write_datasource_legacy(cluster):
    ds = rd.range(25, override_num_blocks=3) if "override_num_blocks" in \
        rd.range.__code__.co_varnames else rd.range(25)
    ds.write_datasource(_Collect())
    src = _LegacySource()
    assert ds.write_datasource(src) == 25 and src.rows == 25


def test_data_iterator_schema_and_to_torch(cluster):
    ds = rd.from_items([{"a": float(i), "b": float(2 * i), "y": i % 2} for i in range(8)])
    it = ds.iterator()
    assert set(it.schema().names) == {"a", "b", "y"}
    batches = list(it.to_torch(label_column="y", feature_columns=["a", "b"], batch_size=4))
    assert len(batches) == 2
    x, y = batches[0]
    assert tuple(x.shape) == (4, 2) and tuple(y.shape) == (4,)


def test_runtime_context_legacy_ids(cluster):
    @ray.remote
    def f():
        ctx = ray.get_runtime_context()
        return ctx.task_id, ctx.get_resource_ids()

    tid, rids = ray.get(f.remote())
    assert isinstance(tid, str) and rids == {"GPU": []}
