"""``BaseTrainer`` (reference: python/ray/train/base_trainer.py).

The base of every trainer. A custom trainer subclasses it and implements
``training_loop()``, calling ``ray_amd.train.report(...)`` (and ``train.get_checkpoint()``
to resume) from inside; ``fit()`` runs that loop in one worker actor with the trainer's
``scaling_config`` resources and returns a ``Result`` with the same run directory,
checkpoint management, callbacks and failure retries as ``DataParallelTrainer`` (which is
itself a BaseTrainer whose loop is spread over ``num_workers`` workers). A trainer passed
to ``Tuner`` runs as one trial per configuration (``as_trainable``)."""

from __future__ import annotations

from typing import Any, Dict, Optional, Union

from ray_amd.air.config import RunConfig, ScalingConfig
from ray_amd.train._checkpoint import Checkpoint

GenDataset = Union["ray_amd.data.Dataset", Any]  # noqa: F821

PREPROCESSOR_DEPRECATION_MESSAGE = (
    "The `preprocessor` argument to Trainers is deprecated: apply the preprocessor to the "
    "datasets before passing them, and save it in the checkpoint's metadata yourself.")


def __getattr__(name):  # TrainingFailedError lives with the trainer machinery
    if name == "TrainingFailedError":
        from ray_amd.train.data_parallel_trainer import TrainingFailedError

        return TrainingFailedError
    raise AttributeError(name)


def _run_training_loop(trainer):
    trainer.setup()
    trainer.training_loop()


class BaseTrainer:
    def __init__(self, *, scaling_config: Optional[ScalingConfig] = None,
                 run_config: Optional[RunConfig] = None,
                 datasets: Optional[Dict[str, GenDataset]] = None,
                 metadata: Optional[Dict[str, Any]] = None,
                 resume_from_checkpoint: Optional[Checkpoint] = None):
        self.scaling_config = scaling_config or ScalingConfig()
        self.run_config = run_config or RunConfig()
        self.datasets = datasets or {}
        self.metadata = metadata or {}
        self.resume_from_checkpoint = resume_from_checkpoint

    # ------------------------------------------------------------------ user hooks
    def setup(self) -> None:
        """Called in the training worker before ``training_loop`` (heavy setup belongs here
        rather than in ``__init__``, which runs on the driver)."""

    def training_loop(self) -> None:
        raise NotImplementedError("a BaseTrainer subclass implements training_loop()")

    def preprocess_datasets(self) -> None:  # deprecated in the reference as well
        raise DeprecationWarning(PREPROCESSOR_DEPRECATION_MESSAGE)

    # ------------------------------------------------------------------ running
    def _as_data_parallel(self):
        from ray_amd.train.data_parallel_trainer import DataParallelTrainer

        sc = self.scaling_config
        one = ScalingConfig(num_workers=1, use_gpu=sc.use_gpu,
                            resources_per_worker=sc.resources_per_worker,
                            trainer_resources=sc.trainer_resources,
                            accelerator_type=sc.accelerator_type)
        trainer = self
        dp = DataParallelTrainer(lambda: _run_training_loop(trainer), scaling_config=one,
                                 run_config=self.run_config,
                                 resume_from_checkpoint=self.resume_from_checkpoint,
                                 metadata=self.metadata)
        return dp

    def fit(self):
        """Run ``training_loop`` in one worker; returns the run's ``Result``."""
        dp = self._as_data_parallel()
        if self.run_config.name is None:
            import copy
            import time

            dp.run_config = copy.copy(self.run_config)
            dp.run_config.name = f"{type(self).__name__}_{time.strftime('%Y-%m-%d_%H-%M-%S')}"
        return dp.fit()

    def as_trainable(self):
        """This trainer as a Tune function trainable (a trial's ``train_loop_config`` /
        ``scaling_config`` entries override the trainer's)."""
        from ray_amd.tune.tuner import _trainer_to_trainable

        return _trainer_to_trainable(self)

    @classmethod
    def can_restore(cls, path) -> bool:
        from ray_amd.train.data_parallel_trainer import DataParallelTrainer

        return DataParallelTrainer.can_restore(path)

    @classmethod
    def restore(cls, path, **kwargs):
        from ray_amd.train.data_parallel_trainer import DataParallelTrainer

        return DataParallelTrainer.restore(path, **kwargs)

    def __repr__(self):
        return f"<{type(self).__name__} scaling_config={self.scaling_config!r}>"
