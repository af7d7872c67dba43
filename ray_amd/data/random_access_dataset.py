"""``ray.data.random_access_dataset`` (reference: python/ray/data/random_access_dataset.py):
``Dataset.to_random_access_dataset(key)`` — a dataset sorted by ``key`` and served by
actors for point lookups (``get_async`` / ``multiget``)."""

from ray_amd.data.datasource import RandomAccessDataset  # noqa: F401

__all__ = ["RandomAccessDataset"]
