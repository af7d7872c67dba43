"""Custom datasources / datasinks and the extra built-in formats.

Reference parity (python/ray/data):
  * ``Datasource`` / ``ReadTask`` (datasource/datasource.py) and ``Datasink``
    (datasource/datasink.py: on_write_start / write / on_write_complete / on_write_failed)
    consumed by ``read_datasource`` and ``Dataset.write_datasink``.
  * ``read_sql`` / ``Dataset.write_sql`` (read_api.py:read_sql, _internal/datasource/
    sql_datasource.py): DB-API 2 connections from a ``connection_factory``; the query is
    sharded with LIMIT/OFFSET over its COUNT(*) so parallel read tasks each pull a slice.
  * ``read_webdataset`` / ``Dataset.write_webdataset`` (webdataset_datasource.py): tar
    shards whose members ``<key>.<ext>`` group into one sample per key, decoded by
    extension (txt/json/cls/npy/images) and encoded back the same way.
  * ``Dataset.write_images`` (image_datasink.py), ``read_parquet_bulk``.
  * ``RandomAccessDataset`` (random_access_dataset.py): the dataset sorted by a key and
    range-partitioned over actors; ``get_async`` / ``multiget`` route by partition bounds
    and binary-search inside the owning actor.
"""

from __future__ import annotations

import io
import json
import os
import tarfile
from typing import Any, Callable, Iterable, List, Optional

import numpy as np

import ray_amd as ray
from ray_amd.data import block as B


# ------------------------------------------------------------------------ API classes
class ReadTask:
    """A zero-argument callable returning one block (or an iterable of blocks), plus
    optional metadata (num_rows, size_bytes, input_files)."""

    def __init__(self, read_fn: Callable[[], Any], metadata: Optional[dict] = None):
        self._read_fn = read_fn
        self.metadata = metadata or {}

    def __call__(self):
        out = self._read_fn()
        if isinstance(out, (list, tuple)) or (hasattr(out, "__next__")):
            blocks = [B.from_batch(b) for b in out]
            return B.concat(blocks) if blocks else {}
        return B.from_batch(out)


class Datasource:
    """Subclass and implement ``get_read_tasks(parallelism) -> list[ReadTask]``."""

    def get_name(self) -> str:
        name = type(self).__name__
        return name[: -len("Datasource")] if name.endswith("Datasource") else name

    def estimate_inmemory_data_size(self) -> Optional[int]:
        return None

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        raise NotImplementedError


class Datasink:
    """Subclass and implement ``write(blocks, ctx)``; it runs once per write task (one
    task per dataset block) and its return values reach ``on_write_complete``."""

    def on_write_start(self) -> None:
        pass

    def write(self, blocks: Iterable[dict], ctx: dict) -> Any:
        raise NotImplementedError

    def on_write_complete(self, write_results: List[Any]) -> Any:
        return None

    def on_write_failed(self, error: Exception) -> None:
        pass

    def get_name(self) -> str:
        name = type(self).__name__
        return name[: -len("Datasink")] if name.endswith("Datasink") else name

    @property
    def supports_distributed_writes(self) -> bool:
        return True


@ray.remote
def _sink_write(sink, blk, idx):
    return sink.write([blk], {"task_idx": idx})


def write_datasink(ds, sink: Datasink, ray_remote_args: Optional[dict] = None):
    from ray_amd.data import _executor as X

    sink.on_write_start()
    fn = _sink_write.options(**ray_remote_args) if ray_remote_args else _sink_write
    try:
        if sink.supports_distributed_writes:
            results = ray.get([fn.remote(sink, r, i)
                               for i, (r, _) in enumerate(X.execute(ds._plan))])
        else:  # single writer in the driver
            results = [sink.write([ray.get(r) for r, _ in X.execute(ds._plan)], {"task_idx": 0})]
    except Exception as e:
        sink.on_write_failed(e)
        raise
    return sink.on_write_complete(results)


# ------------------------------------------------------------------------------- SQL
def _rows_to_block(cursor, rows) -> dict:
    cols = [d[0] for d in cursor.description]
    if not rows:
        return {c: np.array([]) for c in cols}
    return {c: B._col([r[i] for r in rows]) for i, c in enumerate(cols)}


class SQLDatasource(Datasource):
    def __init__(self, sql: str, connection_factory: Callable[[], Any], shard_keys=None):
        self.sql = sql.strip().rstrip(";")
        self.factory = connection_factory

    def _count(self) -> int:
        con = self.factory()
        try:
            cur = con.cursor()
            cur.execute(f"SELECT COUNT(*) FROM ({self.sql}) AS _ray_amd_q")
            return int(cur.fetchone()[0])
        finally:
            con.close()

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        sql, factory = self.sql, self.factory
        n = self._count()
        shards = max(1, min(parallelism, n)) if n else 1

        def task(limit, offset, whole):
            def read():
                con = factory()
                try:
                    cur = con.cursor()
                    if whole:
                        cur.execute(sql)
                    else:
                        cur.execute(f"SELECT * FROM ({sql}) AS _ray_amd_q "
                                    f"LIMIT {limit} OFFSET {offset}")
                    return _rows_to_block(cur, cur.fetchall())
                finally:
                    con.close()
            return ReadTask(read, {"num_rows": limit})

        if shards == 1:
            return [task(n, 0, True)]
        per = -(-n // shards)
        return [task(per, k * per, False) for k in range(shards) if k * per < n]


class SQLDatasink(Datasink):
    """``sql`` is an INSERT with one DB-API placeholder per column (block column order)."""

    def __init__(self, sql: str, connection_factory: Callable[[], Any]):
        self.sql = sql
        self.factory = connection_factory

    def write(self, blocks, ctx):
        con = self.factory()
        n = 0
        try:
            cur = con.cursor()
            for blk in blocks:
                rows = [tuple(B._py(v) for v in r.values()) for r in B.to_rows(blk)]
                if rows:
                    cur.executemany(self.sql, rows)
                    n += len(rows)
            con.commit()
        finally:
            con.close()
        return n

    def on_write_complete(self, write_results):
        return sum(write_results)


def read_sql(sql: str, connection_factory: Callable[[], Any], *, parallelism: int = -1,
             **kw):
    from ray_amd.data.read_api import _parallelism, read_datasource

    return read_datasource(SQLDatasource(sql, connection_factory),
                           parallelism=_parallelism(parallelism) if parallelism else 1)


# ------------------------------------------------------------------------ webdataset
_IMAGE_EXTS = ("png", "jpg", "jpeg", "bmp", "gif", "webp", "ppm", "tif", "tiff")


def _wds_decode(ext: str, data: bytes):
    e = ext.split(".")[-1].lower()
    if e in ("txt", "text"):
        return data.decode("utf-8")
    if e == "json":
        return json.loads(data)
    if e in ("cls", "cls2", "index", "inx", "id"):
        return int(data.decode().strip())
    if e == "npy":
        return np.load(io.BytesIO(data), allow_pickle=False)
    if e in _IMAGE_EXTS:
        from PIL import Image

        return np.asarray(Image.open(io.BytesIO(data)))
    return data


def _wds_encode(ext: str, value) -> bytes:
    e = ext.split(".")[-1].lower()
    if isinstance(value, bytes):
        return value
    if e in ("txt", "text"):
        return str(value).encode()
    if e == "json":
        return json.dumps(B._py(value) if not isinstance(value, (dict, list)) else value).encode()
    if e in ("cls", "cls2", "index", "inx", "id"):
        return str(int(value)).encode()
    if e == "npy":
        buf = io.BytesIO()
        np.save(buf, np.asarray(value), allow_pickle=False)
        return buf.getvalue()
    if e in _IMAGE_EXTS:
        from PIL import Image

        buf = io.BytesIO()
        Image.fromarray(np.asarray(value)).save(buf, format="JPEG" if e == "jpg" else e.upper())
        return buf.getvalue()
    return str(value).encode()


def _split_member(name: str):
    base = os.path.basename(name)
    d = os.path.dirname(name)
    if "." not in base:
        return None, None
    key, ext = base.split(".", 1)
    return (os.path.join(d, key) if d else key), ext


def _read_tar(path: str, decoder: bool, suffixes) -> dict:
    samples: dict = {}
    order = []
    with tarfile.open(path, "r:*") as tf:
        for m in tf:
            if not m.isfile():
                continue
            key, ext = _split_member(m.name)
            if key is None or (suffixes and ext not in suffixes):
                continue
            data = tf.extractfile(m).read()
            if key not in samples:
                samples[key] = {"__key__": key}
                order.append(key)
            samples[key][ext] = _wds_decode(ext, data) if decoder else data
    return B.from_rows([samples[k] for k in order]) if order else {}


def read_webdataset(paths, *, decoder: bool = True, suffixes=None, include_paths=False,
                    **kw):
    from ray_amd.data.read_api import _file_ds

    return _file_ds(paths, [".tar", ".tar.gz", ".tgz"],
                    lambda f: _read_tar(f, decoder, suffixes), include_paths)


@ray.remote
def _write_tar(blk, path, idx, encoder):
    os.makedirs(path, exist_ok=True)
    out = os.path.join(path, f"part_{idx:06d}.tar")
    with tarfile.open(out, "w") as tf:
        for i, row in enumerate(B.to_rows(blk)):
            key = str(row.get("__key__", f"{idx:06d}_{i:06d}"))
            for col, v in row.items():
                if col == "__key__":
                    continue
                data = _wds_encode(col, v) if encoder else (v if isinstance(v, bytes)
                                                             else str(v).encode())
                ti = tarfile.TarInfo(f"{key}.{col}")
                ti.size = len(data)
                tf.addfile(ti, io.BytesIO(data))
    return B.num_rows(blk)


@ray.remote
def _write_images_block(blk, path, column, file_format, idx):
    from PIL import Image

    os.makedirs(path, exist_ok=True)
    imgs = blk[column]
    for i in range(len(imgs)):
        Image.fromarray(np.asarray(imgs[i])).save(
            os.path.join(path, f"{idx:06d}_{i:06d}.{file_format}"))
    return len(imgs)


# ------------------------------------------------------------- random-access dataset
class _RAPartition:
    def __init__(self, blk: dict, key: str):
        self.key = key
        self.blk = blk
        self.keys = np.asarray(blk[key]) if blk else np.array([])

    def get(self, k):
        i = int(np.searchsorted(self.keys, k))
        if i < len(self.keys) and self.keys[i] == k:
            return {c: B._py(v[i]) for c, v in self.blk.items()}
        return None

    def multiget(self, ks):
        return [self.get(k) for k in ks]

    def stats(self):
        return {"num_rows": int(len(self.keys))}


class RandomAccessDataset:
    """Key lookups over a dataset sorted by ``key`` and range-partitioned onto
    ``num_workers`` actors (reference: data/random_access_dataset.py)."""

    def __init__(self, ds, key: str, num_workers: int):
        rows = B.concat([ray.get(r) for r in ds.sort(key).get_internal_block_refs()])
        n = B.num_rows(rows) if rows else 0
        num_workers = max(1, min(num_workers, n or 1))
        per = -(-n // num_workers) if n else 0
        Part = ray.remote(num_cpus=0)(_RAPartition)
        self._key = key
        self._actors, self._lo = [], []
        for w in range(num_workers):
            s, e = w * per, min(n, (w + 1) * per)
            if s >= e and w > 0:
                break
            blk = B.slice_block(rows, s, e) if n else {}
            self._actors.append(Part.remote(blk, key))
            self._lo.append(blk[key][0] if n else None)

    def _owner(self, k) -> int:
        if len(self._actors) == 1 or self._lo[0] is None:
            return 0
        return max(0, int(np.searchsorted(np.asarray(self._lo[1:]), k, side="right")))

    def get_async(self, key):
        return self._actors[self._owner(key)].get.remote(key)

    def multiget(self, keys: List) -> List:
        groups: dict = {}
        for i, k in enumerate(keys):
            groups.setdefault(self._owner(k), []).append(i)
        out: list = [None] * len(keys)
        refs = {a: self._actors[a].multiget.remote([keys[i] for i in idx])
                for a, idx in groups.items()}
        for a, idx in groups.items():
            for i, v in zip(idx, ray.get(refs[a])):
                out[i] = v
        return out

    def stats(self) -> str:
        st = ray.get([a.stats.remote() for a in self._actors])
        return f"RandomAccessDataset: {len(st)} workers, rows per worker " \
               f"{[s['num_rows'] for s in st]}"


# ------------------------------------------------------------ file-based datasinks
class _FileDatasink(Datasink):
    def __init__(self, path: str, *, file_format: str = "bin", filesystem=None,
                 try_create_dir: bool = True, **kw):
        self.path = path
        self.file_format = file_format
        self.try_create_dir = try_create_dir

    def on_write_start(self):
        if self.try_create_dir:
            os.makedirs(self.path, exist_ok=True)

    def _open(self, name: str):
        return open(os.path.join(self.path, name), "wb")


class RowBasedFileDatasink(_FileDatasink):
    """One file per row: implement ``write_row_to_file(row: dict, file)``
    (reference: data/datasource/file_datasink.py RowBasedFileDatasink)."""

    def write_row_to_file(self, row: dict, file) -> None:
        raise NotImplementedError

    def write(self, blocks, ctx):
        n = 0
        for blk in blocks:
            for i, row in enumerate(B.to_rows(blk)):
                with self._open(f"{ctx['task_idx']:06d}_{i:06d}.{self.file_format}") as f:
                    self.write_row_to_file(row, f)
                n += 1
        return n

    def on_write_complete(self, write_results):
        return sum(write_results)


class BlockBasedFileDatasink(_FileDatasink):
    """One file per block: implement ``write_block_to_file(block, file)`` (the block is a
    pyarrow Table, like the reference's BlockAccessor.to_arrow())."""

    def __init__(self, path: str, *, min_rows_per_file: int | None = None, **kw):
        super().__init__(path, **kw)
        self.min_rows_per_file = min_rows_per_file

    def write_block_to_file(self, block, file) -> None:
        raise NotImplementedError

    def write(self, blocks, ctx):
        n = 0
        for j, blk in enumerate(blocks):
            with self._open(f"{ctx['task_idx']:06d}_{j:03d}.{self.file_format}") as f:
                self.write_block_to_file(B.to_batch(blk, "pyarrow"), f)
            n += B.num_rows(blk)
        return n

    def on_write_complete(self, write_results):
        return sum(write_results)
