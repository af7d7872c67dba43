"""WebDataset tar shards (reference: python/ray/data/datasource/webdataset_datasource.py,
webdataset_datasink.py): members ``<key>.<ext>`` group into one sample per key, decoded by
extension (txt/json/cls/npy/images) and encoded back the same way."""

from __future__ import annotations

import io
import json
import os
import tarfile

import numpy as np

import ray_amd as ray
from ray_amd.data import block as B

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
                    filesystem=None, partitioning=None, partition_filter=None, **kw):
    from ray_amd.data.datasource.formats import WebDatasetDatasource
    from ray_amd.data.read_api import read_datasource

    return read_datasource(WebDatasetDatasource(
        paths, decoder=decoder, suffixes=suffixes, include_paths=include_paths,
        filesystem=filesystem, partitioning=partitioning, partition_filter=partition_filter))


def _tar_bytes(blk, idx, encoder) -> bytes:
    """One block as an uncompressed tar shard: row -> members ``<__key__>.<column>``."""
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as tf:
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
    return buf.getvalue()


@ray.remote
def _write_tar(blk, path, idx, encoder):
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, f"part_{idx:06d}.tar"), "wb") as f:
        f.write(_tar_bytes(blk, idx, encoder))
    return B.num_rows(blk)
