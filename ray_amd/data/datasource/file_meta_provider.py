"""File metadata providers (reference: python/ray/data/datasource/file_meta_provider.py,
parquet_meta_provider.py): expand the input paths into (file, size) pairs before reading,
and describe a read task's block."""

from __future__ import annotations

import os
from typing import Iterator, List, Optional, Tuple

from ray_amd.data.datasource.path_util import _expand_local


class FileMetadataProvider:
    def _get_block_metadata(self, paths: List[str], schema=None, *, rows_per_file=None,
                            file_sizes: List[Optional[int]]) -> dict:
        sizes = [s for s in file_sizes if s is not None]
        return {"num_rows": (rows_per_file * len(paths)) if rows_per_file else None,
                "size_bytes": sum(sizes) if len(sizes) == len(file_sizes) else None,
                "schema": schema, "input_files": list(paths)}

    def __call__(self, paths, schema=None, **kwargs) -> dict:
        return self._get_block_metadata(paths, schema, **kwargs)


class BaseFileMetadataProvider(FileMetadataProvider):
    def expand_paths(self, paths: List[str], filesystem=None, partitioning=None,
                     ignore_missing_paths: bool = False) -> Iterator[Tuple[str, Optional[int]]]:
        raise NotImplementedError


class DefaultFileMetadataProvider(BaseFileMetadataProvider):
    """Directories are walked recursively (hidden ``.``/``_`` files skipped), globs
    expanded, and each file's size read."""

    def expand_paths(self, paths, filesystem=None, partitioning=None,
                     ignore_missing_paths: bool = False):
        for p in paths:
            if filesystem is None:
                files = _expand_local(p)
                for f in files:
                    try:
                        yield f, os.path.getsize(f)
                    except FileNotFoundError:
                        if not ignore_missing_paths:
                            raise
            else:
                import pyarrow.fs as pafs

                info = filesystem.get_file_info(p)
                if info.type == pafs.FileType.Directory:
                    sel = pafs.FileSelector(p, recursive=True)
                    for fi in sorted(filesystem.get_file_info(sel), key=lambda x: x.path):
                        base = os.path.basename(fi.path)
                        if fi.type == pafs.FileType.File and base[:1] not in (".", "_"):
                            yield fi.path, fi.size
                elif info.type == pafs.FileType.File:
                    yield p, info.size
                elif not ignore_missing_paths:
                    raise FileNotFoundError(p)


class FastFileMetadataProvider(DefaultFileMetadataProvider):
    """Skips the per-file size lookup (sizes unknown): fastest for many small local files."""

    def expand_paths(self, paths, filesystem=None, partitioning=None,
                     ignore_missing_paths: bool = False):
        if filesystem is not None:
            yield from super().expand_paths(paths, filesystem, partitioning,
                                            ignore_missing_paths)
            return
        for p in paths:
            for f in _expand_local(p):
                yield f, None


class ParquetMetadataProvider(FileMetadataProvider):
    def prefetch_file_metadata(self, fragments, **ray_remote_args):
        """Parquet footers of ``fragments`` (pyarrow ParquetFileFragment), or None."""
        return None


class DefaultParquetMetadataProvider(ParquetMetadataProvider):
    def prefetch_file_metadata(self, fragments, **ray_remote_args):
        return [f.metadata for f in fragments]
