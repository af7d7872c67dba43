"""``ray.train.context`` (reference: python/ray/train/context.py): the per-worker
``TrainContext`` (ranks, world size, trial info, storage) and ``get_context()``."""

from ray_amd.train._internal.session import TrainContext, get_context  # noqa: F401

__all__ = ["TrainContext", "get_context"]
