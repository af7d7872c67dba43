"""``Datasource`` / ``ReadTask`` (reference: python/ray/data/datasource/datasource.py).

A datasource turns into read tasks (``get_read_tasks(parallelism)``); each task is a
zero-argument callable returning one block, or an iterable of blocks, run as one Ray task
of the dataset's read stage (``read_api.read_datasource``)."""

from __future__ import annotations

from typing import Any, Callable, List, Optional

from ray_amd.data import block as B


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


class Reader:
    """The reference's deprecated reader object: ``get_read_tasks(parallelism)``."""

    def estimate_inmemory_data_size(self) -> Optional[int]:
        return None

    def get_read_tasks(self, parallelism: int) -> List[ReadTask]:
        raise NotImplementedError
