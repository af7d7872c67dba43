"""Dataset sources (reference: python/ray/data/read_api.py, datasource/*)."""

from __future__ import annotations

import os

import numpy as np

import ray_amd as ray

from . import _executor as X
from . import block as B
from .dataset import Dataset, MaterializedDataset


def _parallelism(p, n_items=None):
    if p in (None, -1, "auto"):
        p = X.default_parallelism() * 2
    if n_items is not None:
        p = max(1, min(p, n_items))
    return int(p)


def range(n: int, *, parallelism: int = -1, override_num_blocks=None) -> Dataset:  # noqa: A001
    k = _parallelism(override_num_blocks or parallelism, n)
    bounds = [n * i // k for i in builtins_range(k + 1)]

    def mk(lo, hi):
        return lambda: {"id": np.arange(lo, hi, dtype=np.int64)}

    return Dataset(X.Plan(("read", [mk(bounds[i], bounds[i + 1]) for i in builtins_range(k)])))


def range_tensor(n: int, *, shape=(1,), parallelism: int = -1, override_num_blocks=None):
    k = _parallelism(override_num_blocks or parallelism, n)
    bounds = [n * i // k for i in builtins_range(k + 1)]

    def mk(lo, hi):
        def f():
            ids = np.arange(lo, hi, dtype=np.int64)
            return {"data": np.broadcast_to(ids.reshape((-1,) + (1,) * len(shape)),
                                            (hi - lo,) + tuple(shape)).copy()}
        return f

    return Dataset(X.Plan(("read", [mk(bounds[i], bounds[i + 1]) for i in builtins_range(k)])))


def from_items(items: list, *, parallelism: int = -1, override_num_blocks=None) -> Dataset:
    k = _parallelism(override_num_blocks or parallelism, max(1, len(items)))
    bounds = [len(items) * i // k for i in builtins_range(k + 1)]
    refs, metas = [], []
    for i in builtins_range(k):
        blk = B.from_rows(items[bounds[i]:bounds[i + 1]])
        refs.append(ray.put(blk))
        metas.append(X._meta(blk))
    return MaterializedDataset(X.Plan(("refs", refs), source_meta=metas))


def _from_blocks(blocks):
    refs = [ray.put(b) for b in blocks]
    return MaterializedDataset(X.Plan(("refs", refs), source_meta=[X._meta(b) for b in blocks]))


def from_numpy(ndarrays) -> Dataset:
    if isinstance(ndarrays, np.ndarray):
        ndarrays = [ndarrays]
    return _from_blocks([{"data": a} for a in ndarrays])


def from_numpy_refs(refs) -> Dataset:
    return _from_blocks([{"data": ray.get(r)} for r in refs])


def from_pandas(dfs) -> Dataset:
    if not isinstance(dfs, list):
        dfs = [dfs]
    return _from_blocks([B.from_batch(d) for d in dfs])


def from_pandas_refs(refs):
    return from_pandas([ray.get(r) for r in refs])


def from_arrow(tables) -> Dataset:
    if not isinstance(tables, list):
        tables = [tables]
    return _from_blocks([B.from_batch(t) for t in tables])


def from_arrow_refs(refs):
    return from_arrow([ray.get(r) for r in refs])


def from_torch(dataset) -> Dataset:
    return from_items([{"item": dataset[i]} for i in builtins_range(len(dataset))])


def from_huggingface(dataset) -> Dataset:
    return from_items([dict(r) for r in dataset])


_FILE_KW = ("filesystem", "schema", "open_stream_args", "arrow_open_stream_args",
            "meta_provider", "partition_filter", "partitioning", "ignore_missing_paths",
            "shuffle", "include_paths", "file_extensions")


def _file_kw(kw: dict, partitioning_default="hive") -> dict:
    """The FileBasedDatasource keywords of a read_* call (the rest are format options)."""
    out = {k: kw.pop(k) for k in list(kw) if k in _FILE_KW}
    if "arrow_open_stream_args" in out:
        out["open_stream_args"] = out.pop("arrow_open_stream_args")
    out.setdefault("partitioning", partitioning_default)
    for k in ("parallelism", "override_num_blocks", "ray_remote_args", "concurrency",
              "tensor_column_schema", "dataset_kwargs"):
        kw.pop(k, None)
    return out


def read_parquet(paths, *, columns=None, **kw) -> Dataset:
    from ray_amd.data.datasource.formats import ParquetDatasource

    return read_datasource(ParquetDatasource(paths, columns=columns, **_file_kw(kw)))


def read_csv(paths, **kw) -> Dataset:
    from ray_amd.data.datasource.formats import CSVDatasource

    fkw = _file_kw(kw)
    return read_datasource(CSVDatasource(paths, arrow_csv_args=kw, **fkw))


def read_json(paths, *, lines=None, **kw) -> Dataset:
    from ray_amd.data.datasource.formats import JSONDatasource

    return read_datasource(JSONDatasource(paths, lines=lines, **_file_kw(kw)))


def read_numpy(paths, **kw) -> Dataset:
    from ray_amd.data.datasource.formats import NumpyDatasource

    return read_datasource(NumpyDatasource(paths, **_file_kw(kw, None)))


def read_text(paths, *, encoding="utf-8", drop_empty_lines=True, **kw):
    from ray_amd.data.datasource.formats import TextDatasource

    return read_datasource(TextDatasource(paths, drop_empty_lines=drop_empty_lines,
                                          encoding=encoding, **_file_kw(kw, None)))


def read_tfrecords(paths, *, tf_schema=None, verify=True, **kw) -> Dataset:
    """TFRecord files of tf.train.Example protos (data/tfrecords.py); one block per file.
    ``verify`` checks every record's CRC32C; ``arrow_open_stream_args={"compression":
    "gzip"}`` (or a ``.gz`` suffix) reads compressed files."""
    from ray_amd.data.datasource.formats import TFRecordDatasource

    return read_datasource(TFRecordDatasource(paths, tf_schema=tf_schema, verify=verify,
                                              **_file_kw(kw, None)))


def read_avro(paths, **kw) -> Dataset:
    """Avro object container files (data/avro.py): one block per file, a column per
    top-level record field."""
    from ray_amd.data.datasource.formats import AvroDatasource

    return read_datasource(AvroDatasource(paths, **_file_kw(kw, None)))


def read_binary_files(paths, **kw) -> Dataset:
    from ray_amd.data.datasource.formats import BinaryDatasource

    return read_datasource(BinaryDatasource(paths, **_file_kw(kw, None)))


def read_images(paths, *, size=None, mode=None, **kw) -> Dataset:
    """Image files (png/jpg/bmp/gif/webp/tiff via PIL, or .npy HWC arrays) -> rows with an
    ``image`` HWC uint8 array; ``size=(h, w)`` resizes, ``mode`` converts (e.g. "RGB")."""
    from ray_amd.data.datasource.formats import ImageDatasource

    return read_datasource(ImageDatasource(paths, size=size, mode=mode,
                                           **_file_kw(kw, None)))


def read_parquet_bulk(paths, *, columns=None, **kw) -> Dataset:
    """read_parquet over an explicit file list (no metadata pass; sizes not fetched)."""
    from ray_amd.data.datasource.file_meta_provider import FastFileMetadataProvider

    kw.setdefault("meta_provider", FastFileMetadataProvider())
    return read_parquet(list(paths) if not isinstance(paths, str) else [paths],
                        columns=columns, **kw)


def read_datasource(datasource, *, parallelism=-1, override_num_blocks=None,
                    **kw) -> Dataset:
    p = override_num_blocks if override_num_blocks is not None else parallelism
    tasks = datasource.get_read_tasks(_parallelism(p))
    ds = Dataset(X.Plan(("read", list(tasks))))
    if hasattr(datasource, "input_files"):
        ds._input_files = datasource.input_files()
    return ds


import builtins  # noqa: E402

builtins_range = builtins.range
