"""Output file names of file writes (reference: python/ray/data/datasource/
filename_provider.py)."""

from __future__ import annotations

from typing import Any, Dict, Optional


class FilenameProvider:
    """Implement ``get_filename_for_block`` (one file per block) and/or
    ``get_filename_for_row`` (one file per row)."""

    def get_filename_for_block(self, block, task_index: int, block_index: int) -> str:
        raise NotImplementedError

    def get_filename_for_row(self, row: Dict[str, Any], task_index: int, block_index: int,
                             row_index: int) -> str:
        raise NotImplementedError


class _DefaultFilenameProvider(FilenameProvider):
    def __init__(self, dataset_uuid: Optional[str] = None, file_format: Optional[str] = None):
        self._uuid = dataset_uuid
        self._ext = file_format

    def _name(self, stem: str) -> str:
        if self._uuid:
            stem = f"{self._uuid}_{stem}"
        return f"{stem}.{self._ext}" if self._ext else stem

    def get_filename_for_block(self, block, task_index, block_index):
        return self._name(f"{task_index:06d}_{block_index:06d}")

    def get_filename_for_row(self, row, task_index, block_index, row_index):
        return self._name(f"{task_index:06d}_{block_index:06d}_{row_index:06d}")
