"""``ray.tune.syncer`` (reference: python/ray/tune/syncer.py): ``SyncConfig``. Run
directories are written straight to ``RunConfig.storage_path`` (a local path or a pyarrow
filesystem URI, train/_internal/storage.py), so there is no separate syncer process."""

from ray_amd.air.config import SyncConfig  # noqa: F401

__all__ = ["SyncConfig"]
