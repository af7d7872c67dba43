"""``ray.train.trainer`` (reference: python/ray/train/trainer.py): ``TrainingIterator``,
iterating a trainer's reports as they arrive."""

from ray_amd.train.data_parallel_trainer import TrainingIterator  # noqa: F401

__all__ = ["TrainingIterator"]
