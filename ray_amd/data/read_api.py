"""Dataset sources (reference: python/ray/data/read_api.py, datasource/*)."""

from __future__ import annotations

import glob
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


def _expand(paths, exts=None):
    if isinstance(paths, str):
        paths = [paths]
    out = []
    for p in paths:
        if os.path.isdir(p):
            for root, _, files in os.walk(p):
                for f in sorted(files):
                    if exts is None or any(f.endswith(e) for e in exts):
                        out.append(os.path.join(root, f))
        elif any(c in p for c in "*?["):
            out.extend(sorted(glob.glob(p)))
        else:
            out.append(p)
    if not out:
        raise FileNotFoundError(f"no files found for {paths}")
    return out


def _hive_values(f: str, paths) -> dict:
    """``key=value`` directory segments between an input directory and the file
    (reference: datasource/partitioning.py Partitioning("hive")); values stay strings."""
    out = {}
    for p in ([paths] if isinstance(paths, str) else paths):
        p = os.path.abspath(p)
        af = os.path.abspath(f)
        if os.path.isdir(p) and af.startswith(p.rstrip(os.sep) + os.sep):
            for seg in os.path.relpath(os.path.dirname(af), p).split(os.sep):
                k, sep, v = seg.partition("=")
                if sep and k:
                    out[k] = v
            break
    return out


def _file_ds(paths, exts, reader, include_paths=False, partitioning="hive",
             partition_filter=None):
    files = _expand(paths, exts)
    parts = {f: (_hive_values(f, paths) if partitioning == "hive" else {}) for f in files}
    if partition_filter is not None:
        files = [f for f in files if partition_filter(parts[f])]
        if not files:
            raise FileNotFoundError(f"partition_filter kept no files of {paths}")

    def mk(f):
        def r():
            blk = B.from_batch(reader(f))
            n = B.num_rows(blk)
            for k, v in parts[f].items():
                if k not in blk:
                    blk[k] = np.array([v] * n, dtype=object)
            if include_paths:
                blk["path"] = np.array([f] * B.num_rows(blk), dtype=object)
            return blk
        return r

    ds = Dataset(X.Plan(("read", [mk(f) for f in files])))
    ds._input_files = files
    return ds


def read_parquet(paths, *, columns=None, include_paths=False, partitioning="hive",
                 partition_filter=None, **kw) -> Dataset:
    def rd(f):
        import pyarrow.parquet as pq

        # tensor extension columns (ray.data.arrow_tensor) must be registered in the
        # reading process, or they load as plain lists
        from ray_amd.data.extensions import tensor_extension  # noqa: F401

        return pq.read_table(f, columns=columns, partitioning=None)

    return _file_ds(paths, [".parquet"], rd, include_paths, partitioning, partition_filter)


def read_csv(paths, *, include_paths=False, partitioning="hive", partition_filter=None,
             **kw) -> Dataset:
    def rd(f):
        import pyarrow.csv as pc

        return pc.read_csv(f)

    return _file_ds(paths, [".csv"], rd, include_paths, partitioning, partition_filter)


def read_json(paths, *, include_paths=False, lines=True, partitioning="hive",
              partition_filter=None, **kw) -> Dataset:
    def rd(f):
        import pandas as pd

        try:
            return pd.read_json(f, lines=True)
        except ValueError:
            return pd.read_json(f)

    return _file_ds(paths, [".json", ".jsonl"], rd, include_paths, partitioning,
                    partition_filter)


def read_numpy(paths, *, include_paths=False, **kw) -> Dataset:
    return _file_ds(paths, [".npy"], lambda f: {"data": np.load(f)}, include_paths)


def read_text(paths, *, encoding="utf-8", drop_empty_lines=True, include_paths=False, **kw):
    def rd(f):
        with open(f, encoding=encoding) as fh:
            lines = [ln.rstrip("\n") for ln in fh]
        if drop_empty_lines:
            lines = [ln for ln in lines if ln.strip()]
        return {"text": np.array(lines, dtype=object)}

    return _file_ds(paths, None, rd, include_paths)


def read_tfrecords(paths, *, include_paths=False, tf_schema=None, verify=True,
                   arrow_open_stream_args=None, **kw) -> Dataset:
    """TFRecord files of tf.train.Example protos (data/tfrecords.py); one block per file.
    ``verify`` checks every record's CRC32C; ``arrow_open_stream_args={"compression":
    "gzip"}`` (or a ``.gz`` suffix) reads compressed files."""
    from ray_amd.data.tfrecords import read_file

    if tf_schema is not None:
        raise NotImplementedError("tf_schema needs tensorflow_metadata (not installed)")
    comp = (arrow_open_stream_args or {}).get("compression")
    return _file_ds(paths, [".tfrecords", ".tfrecord", ".gz"],
                    lambda f: read_file(f, verify, comp), include_paths)


def read_avro(paths, *, include_paths=False, **kw) -> Dataset:
    """Avro object container files (data/avro.py): one block per file, a column per
    top-level record field."""
    from ray_amd.data.avro import read_file

    return _file_ds(paths, [".avro"], read_file, include_paths)


def read_binary_files(paths, *, include_paths=False, **kw) -> Dataset:
    def rd(f):
        with open(f, "rb") as fh:
            b = np.empty(1, dtype=object)
            b[0] = fh.read()
        return {"bytes": b}

    return _file_ds(paths, None, rd, include_paths)


def read_images(paths, *, size=None, mode=None, include_paths=False, **kw) -> Dataset:
    """Image files (png/jpg/bmp/gif/webp/tiff via PIL, or .npy HWC arrays) -> rows with an
    ``image`` HWC uint8 array; ``size=(h, w)`` resizes, ``mode`` converts (e.g. "RGB")."""
    exts = [".png", ".jpg", ".jpeg", ".bmp", ".gif", ".webp", ".tif", ".tiff", ".npy"]

    def rd(f):
        if f.endswith(".npy"):
            img = np.load(f)
        else:
            from PIL import Image

            im = Image.open(f)
            if mode is not None:
                im = im.convert(mode)
            if size is not None:
                im = im.resize((size[1], size[0]))
            img = np.asarray(im)
        return {"image": img[None]}

    return _file_ds(paths, exts, rd, include_paths)


def read_parquet_bulk(paths, *, columns=None, include_paths=False, **kw) -> Dataset:
    """read_parquet over an explicit file list (no directory expansion / metadata pass)."""
    return read_parquet(list(paths) if not isinstance(paths, str) else [paths],
                        columns=columns, include_paths=include_paths)


def read_datasource(datasource, *, parallelism=-1, **kw) -> Dataset:
    tasks = datasource.get_read_tasks(_parallelism(parallelism))
    return Dataset(X.Plan(("read", list(tasks))))


import builtins  # noqa: E402

builtins_range = builtins.range
