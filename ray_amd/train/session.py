"""``ray.train.session`` (reference: python/ray/train/session.py, a compatibility module):
the session functions a training loop calls."""

from ray_amd.train._internal.session import (get_checkpoint, get_context,  # noqa: F401
                                             get_dataset_shard, report)

__all__ = ["get_checkpoint", "get_context", "get_dataset_shard", "report"]
