"""In-memory and service-backed datasources (reference: python/ray/data/datasource/
{range,torch,huggingface,mongo,bigquery,databricks_uc}_datasource.py and the
``RandomIntRowDatasource`` test source)."""

from __future__ import annotations

from typing import List, Optional

import numpy as np

from ray_amd.data.datasource.datasource import Datasource, ReadTask


class RangeDatasource(Datasource):
    """Integers 0..n-1 as column ``column_name`` (or an ``(n, *shape)`` tensor column with
    ``block_format="tensor"``)."""

    def __init__(self, n: int, block_format: str = "arrow", tensor_shape=(1,),
                 column_name: Optional[str] = None):
        self._n = int(n)
        self._format = block_format
        self._shape = tuple(tensor_shape)
        self._col = column_name or ("data" if block_format == "tensor" else "id")

    def estimate_inmemory_data_size(self):
        return self._n * 8 * (int(np.prod(self._shape)) if self._format == "tensor" else 1)

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        n, par = self._n, max(1, min(parallelism, self._n or 1))
        per = -(-n // par) if n else 0
        col, fmt, shape = self._col, self._format, self._shape
        tasks = []
        for s in range(0, n, per or 1):
            e = min(n, s + per)

            def read(s=s, e=e):
                ids = np.arange(s, e, dtype=np.int64)
                if fmt == "tensor":
                    return {col: np.broadcast_to(ids.reshape((-1,) + (1,) * len(shape)),
                                                 (e - s,) + shape).copy()}
                return {col: ids}
            tasks.append(ReadTask(read, {"num_rows": e - s}))
            if per == 0:
                break
        return tasks


class RandomIntRowDatasource(Datasource):
    """``n`` rows of ``num_columns`` random int64 columns ``c_0..``."""

    def __init__(self, n: int, num_columns: int, seed: Optional[int] = None):
        self._n, self._cols, self._seed = int(n), int(num_columns), seed

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        n, par = self._n, max(1, min(parallelism, self._n or 1))
        per = -(-n // par)
        tasks = []
        for i, s in enumerate(range(0, n, per)):
            e = min(n, s + per)

            def read(s=s, e=e, i=i):
                rng = np.random.default_rng(None if self._seed is None else self._seed + i)
                return {f"c_{j}": rng.integers(0, 2 ** 31, e - s, dtype=np.int64)
                        for j in range(self._cols)}
            tasks.append(ReadTask(read, {"num_rows": e - s}))
        return tasks


class TorchDatasource(Datasource):
    """A map-style ``torch.utils.data.Dataset`` as rows ``{"item": dataset[i]}``, read in
    ``parallelism`` index ranges."""

    def __init__(self, dataset):
        self._ds = dataset

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        n = len(self._ds)
        par = max(1, min(parallelism, n or 1))
        per = -(-n // par) if n else 0
        ds = self._ds
        tasks = []
        for s in range(0, n, per or 1):
            e = min(n, s + per)

            def read(s=s, e=e):
                items = np.empty(e - s, dtype=object)
                for j, i in enumerate(range(s, e)):
                    items[j] = ds[i]
                return {"item": items}
            tasks.append(ReadTask(read, {"num_rows": e - s}))
            if per == 0:
                break
        return tasks


class HuggingFaceDatasource(Datasource):
    """A ``datasets.Dataset`` (arrow-backed) split into ``parallelism`` row ranges."""

    def __init__(self, dataset, batch_size: int = 4096):
        self._ds = dataset

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        n = len(self._ds)
        par = max(1, min(parallelism, n or 1))
        per = -(-n // par) if n else 0
        tbl = self._ds.with_format("arrow")[:] if hasattr(self._ds, "with_format") else None
        tasks = []
        for s in range(0, n, per or 1):
            e = min(n, s + per)

            def read(s=s, e=e):
                if tbl is not None:
                    return tbl.slice(s, e - s)
                return [dict(self._ds[i]) for i in range(s, e)]
            tasks.append(ReadTask(read, {"num_rows": e - s}))
            if per == 0:
                break
        return tasks


class MongoDatasource(Datasource):
    """A MongoDB collection (``pymongo``), read in one task per ``_id`` range of the
    given pipeline's output."""

    def __init__(self, uri: str, database: str, collection: str, pipeline=None,
                 schema=None, **mongo_args):
        self._uri, self._db, self._coll = uri, database, collection
        self._pipeline = pipeline or []
        self._args = mongo_args

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        from ray_amd.data import integrations

        ds = integrations.read_mongo(self._uri, self._db, self._coll,
                                     pipeline=self._pipeline, parallelism=parallelism,
                                     **self._args)
        return [ReadTask(lambda r=r: __import__("ray_amd").get(r))
                for r in ds.get_internal_block_refs()]


class BigQueryDatasource(Datasource):
    def __init__(self, project_id: str, dataset: Optional[str] = None,
                 query: Optional[str] = None):
        try:
            from google.cloud import bigquery  # noqa: F401
        except ImportError as e:
            raise ImportError("BigQueryDatasource needs 'google-cloud-bigquery', which is "
                              "not installed") from e
        self._project, self._dataset, self._query = project_id, dataset, query

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        from ray_amd.data import integrations

        ds = integrations.read_bigquery(self._project, self._dataset, query=self._query)
        return [ReadTask(lambda r=r: __import__("ray_amd").get(r))
                for r in ds.get_internal_block_refs()]


class DatabricksUCDatasource(Datasource):
    def __init__(self, host: str, token: str, warehouse_id: str, catalog: str, schema: str,
                 query: str):
        raise ImportError("the Databricks Unity Catalog reader needs network access to a "
                          "Databricks SQL warehouse (read_databricks_tables)")
