"""File datasinks (reference: python/ray/data/datasource/file_datasink.py and the format
sinks csv/json/parquet/numpy/image/tfrecords/webdataset_datasink.py).

``RowBasedFileDatasink`` writes one file per row (``write_row_to_file``),
``BlockBasedFileDatasink`` one file per block (``write_block_to_file``, the block as a
pyarrow Table). File names come from a ``FilenameProvider`` (default
``<dataset uuid>_<task>_<block>.<format>``); ``filesystem`` may be any pyarrow filesystem
(or the path a URI)."""

from __future__ import annotations

import os
import uuid
from typing import Any, Dict, Optional

import numpy as np

from ray_amd.data import block as B
from ray_amd.data.datasource.datasink import Datasink
from ray_amd.data.datasource.filename_provider import FilenameProvider, _DefaultFilenameProvider
from ray_amd.data.datasource.path_util import _resolve_paths_and_filesystem


class _FileDatasink(Datasink):
    def __init__(self, path: str, *, filesystem=None, try_create_dir: bool = True,
                 open_stream_args: Optional[Dict[str, Any]] = None,
                 filename_provider: Optional[FilenameProvider] = None,
                 dataset_uuid: Optional[str] = None, file_format: Optional[str] = None,
                 block_path_provider=None, **kw):
        (self.path,), self.filesystem = _resolve_paths_and_filesystem(path, filesystem)
        self.try_create_dir = try_create_dir
        self.open_stream_args = dict(open_stream_args or {})
        self.file_format = file_format or getattr(self, "_FORMAT", "bin")
        self.dataset_uuid = dataset_uuid or uuid.uuid4().hex[:12]
        self.filename_provider = filename_provider or _DefaultFilenameProvider(
            self.dataset_uuid, self.file_format)
        self.block_path_provider = block_path_provider
        self.has_created_dir = False

    def on_write_start(self):
        if self.try_create_dir:
            if self.filesystem is None:
                os.makedirs(self.path, exist_ok=True)
            else:
                self.filesystem.create_dir(self.path, recursive=True)
            self.has_created_dir = True

    def _open(self, name: str):
        full = os.path.join(self.path, name) if self.filesystem is None else \
            f"{self.path.rstrip('/')}/{name}"
        if self.filesystem is None:
            os.makedirs(os.path.dirname(full), exist_ok=True)
            return open(full, "wb")
        return self.filesystem.open_output_stream(full, **self.open_stream_args)

    def on_write_complete(self, write_results):
        return sum(r for r in write_results if isinstance(r, int))


class RowBasedFileDatasink(_FileDatasink):
    """One file per row: implement ``write_row_to_file(row: dict, file)``."""

    def write_row_to_file(self, row: dict, file) -> None:
        raise NotImplementedError

    def write(self, blocks, ctx):
        n = 0
        for j, blk in enumerate(blocks):
            for i, row in enumerate(B.to_rows(blk)):
                name = self.filename_provider.get_filename_for_row(row, ctx["task_idx"], j, i)
                with self._open(name) as f:
                    self.write_row_to_file(row, f)
                n += 1
        return n


class BlockBasedFileDatasink(_FileDatasink):
    """One file per block: implement ``write_block_to_file(block, file)`` (the block is a
    pyarrow Table, like the reference's BlockAccessor.to_arrow())."""

    def __init__(self, path: str, *, min_rows_per_file: Optional[int] = None, **kw):
        super().__init__(path, **kw)
        self.min_rows_per_file = min_rows_per_file

    def write_block_to_file(self, block, file) -> None:
        raise NotImplementedError

    def write(self, blocks, ctx):
        blocks = [b for b in blocks if b and B.num_rows(b)]
        if self.min_rows_per_file and len(blocks) > 1:
            blocks = [B.concat(blocks)]
        n = 0
        for j, blk in enumerate(blocks):
            name = self.filename_provider.get_filename_for_block(blk, ctx["task_idx"], j)
            with self._open(name) as f:
                self.write_block_to_file(B.to_batch(blk, "pyarrow"), f)
            n += B.num_rows(blk)
        return n


# ---------------------------------------------------------------- format datasinks
class _ParquetDatasink(BlockBasedFileDatasink):
    _FORMAT = "parquet"

    def __init__(self, path, *, arrow_parquet_args: Optional[dict] = None, **kw):
        super().__init__(path, **kw)
        self.arrow_parquet_args = dict(arrow_parquet_args or {})

    def write_block_to_file(self, block, file):
        import pyarrow.parquet as pq

        pq.write_table(block, file, **self.arrow_parquet_args)


class _CSVDatasink(BlockBasedFileDatasink):
    _FORMAT = "csv"

    def __init__(self, path, *, arrow_csv_args: Optional[dict] = None, **kw):
        super().__init__(path, **kw)
        self.arrow_csv_args = dict(arrow_csv_args or {})

    def write_block_to_file(self, block, file):
        import pyarrow.csv as pc

        pc.write_csv(block, file, **self.arrow_csv_args)


class _JSONDatasink(BlockBasedFileDatasink):
    _FORMAT = "json"

    def __init__(self, path, *, pandas_json_args: Optional[dict] = None, **kw):
        super().__init__(path, **kw)
        self.pandas_json_args = dict(pandas_json_args or {})
        self.pandas_json_args.setdefault("orient", "records")
        self.pandas_json_args.setdefault("lines", True)

    def write_block_to_file(self, block, file):
        file.write(block.to_pandas().to_json(**self.pandas_json_args).encode())


class _NumpyDatasink(BlockBasedFileDatasink):
    _FORMAT = "npy"

    def __init__(self, path, column: str, **kw):
        super().__init__(path, **kw)
        self.column = column

    def write(self, blocks, ctx):
        n = 0
        for j, blk in enumerate(b for b in blocks if b and B.num_rows(b)):
            name = self.filename_provider.get_filename_for_block(blk, ctx["task_idx"], j)
            with self._open(name) as f:
                np.save(f, np.asarray(blk[self.column]), allow_pickle=False)
            n += B.num_rows(blk)
        return n


class _ImageDatasink(RowBasedFileDatasink):
    def __init__(self, path, column: str, file_format: str = "png", **kw):
        super().__init__(path, file_format=file_format, **kw)
        self.column = column

    def write_row_to_file(self, row, file):
        from PIL import Image

        Image.fromarray(np.asarray(row[self.column])).save(
            file, format="JPEG" if self.file_format in ("jpg", "jpeg") else
            self.file_format.upper())


class _TFRecordDatasink(BlockBasedFileDatasink):
    _FORMAT = "tfrecords"

    def write_block_to_file(self, block, file):
        from ray_amd.data import tfrecords as T

        file.write(T.encode_block(B.from_batch(block)))


class _WebDatasetDatasink(BlockBasedFileDatasink):
    _FORMAT = "tar"

    def __init__(self, path, encoder: bool = True, **kw):
        super().__init__(path, **kw)
        self.encoder = encoder

    def write_block_to_file(self, block, file):
        from ray_amd.data.datasource.webdataset_datasource import _tar_bytes

        file.write(_tar_bytes(B.from_batch(block), 0, self.encoder))
