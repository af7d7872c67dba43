"""Low-level workflow storage (reference: python/ray/workflow/storage/{__init__,base}.py):
the key/value primitives the workflow layer persists step outputs through, plus a
filesystem implementation (the storage ``workflow.init(storage=<dir>)`` writes to)."""

from __future__ import annotations

import abc
import json
import os
import pickle
import shutil
from typing import Any, List


class DataLoadError(Exception):
    pass


class DataSaveError(Exception):
    pass


class KeyNotFoundError(KeyError):
    pass


class Storage(metaclass=abc.ABCMeta):
    """Async key/value interface: ``put`` / ``get`` / ``delete_prefix`` /
    ``scan_prefix`` over "/"-joined keys."""

    def make_key(self, *names: str) -> str:
        return "/".join(names)

    @abc.abstractmethod
    async def put(self, key: str, data: Any, is_json: bool = False) -> None:
        """Store ``data`` at ``key`` (JSON text or a pickle)."""

    @abc.abstractmethod
    async def get(self, key: str, is_json: bool = False) -> Any:
        """The value at ``key``; KeyNotFoundError if absent."""

    @abc.abstractmethod
    async def delete_prefix(self, key_prefix: str) -> None:
        """Remove every key under ``key_prefix``."""

    @abc.abstractmethod
    async def scan_prefix(self, key_prefix: str) -> List[str]:
        """The names directly under ``key_prefix``."""

    @property
    @abc.abstractmethod
    def storage_url(self) -> str:
        """The URL this storage was created from."""


class FilesystemStorage(Storage):
    """Keys are paths under a root directory; writes go through a temp file + rename."""

    def __init__(self, root: str):
        self._root = os.path.abspath(os.path.expanduser(root))
        os.makedirs(self._root, exist_ok=True)

    def _path(self, key):
        return os.path.join(self._root, *key.split("/"))

    async def put(self, key, data, is_json=False):
        p = self._path(key)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        tmp = p + ".tmp"
        try:
            if is_json:
                with open(tmp, "w") as f:
                    json.dump(data, f)
            else:
                with open(tmp, "wb") as f:
                    pickle.dump(data, f)
            os.replace(tmp, p)
        except Exception as e:  # noqa: BLE001
            raise DataSaveError(f"saving {key}: {e}") from e

    async def get(self, key, is_json=False):
        p = self._path(key)
        if not os.path.exists(p):
            raise KeyNotFoundError(key)
        try:
            if is_json:
                with open(p) as f:
                    return json.load(f)
            with open(p, "rb") as f:  # this storage's own files (written by put)
                return pickle.load(f)
        except Exception as e:  # noqa: BLE001
            raise DataLoadError(f"loading {key}: {e}") from e

    async def delete_prefix(self, key_prefix):
        p = self._path(key_prefix)
        if os.path.isdir(p):
            shutil.rmtree(p)
        elif os.path.exists(p):
            os.unlink(p)

    async def scan_prefix(self, key_prefix):
        p = self._path(key_prefix)
        return sorted(os.listdir(p)) if os.path.isdir(p) else []

    @property
    def storage_url(self):
        return "file://" + self._root


__all__ = ("Storage", "DataLoadError", "DataSaveError", "KeyNotFoundError",
           "FilesystemStorage")
