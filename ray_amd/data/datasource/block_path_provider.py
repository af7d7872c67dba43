"""The reference's deprecated write-path providers (python/ray/data/datasource/
block_path_provider.py); new code passes a ``FilenameProvider``."""

from __future__ import annotations

import posixpath
from typing import Optional


class BlockWritePathProvider:
    def _get_write_path_for_block(self, base_path: str, *, filesystem=None,
                                  dataset_uuid: Optional[str] = None, task_index=None,
                                  block_index=None, file_format=None) -> str:
        raise NotImplementedError

    def __call__(self, base_path, **kwargs) -> str:
        return self._get_write_path_for_block(base_path, **kwargs)


class DefaultBlockWritePathProvider(BlockWritePathProvider):
    def _get_write_path_for_block(self, base_path, *, filesystem=None, dataset_uuid=None,
                                  task_index=None, block_index=None, file_format=None):
        name = f"{dataset_uuid}_{task_index:06d}_{block_index:06d}.{file_format}"
        return posixpath.join(base_path, name)
