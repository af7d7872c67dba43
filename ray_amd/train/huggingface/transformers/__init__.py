"""Hugging Face ``transformers.Trainer`` inside ray_amd Train workers (reference:
python/ray/train/huggingface/transformers/_transformers_utils.py).

Usage inside a ``TorchTrainer`` ``train_loop_per_worker`` (each worker already has
its process group — RCCL on MI355X, gloo on CPU — so ``transformers`` sees a
launched distributed job and wraps the model in DDP itself):

    trainer = transformers.Trainer(model=..., args=..., train_dataset=shard_iterable)
    trainer.add_callback(RayTrainReportCallback())
    trainer = prepare_trainer(trainer)
    trainer.train()

``RayTrainReportCallback`` turns every HF checkpoint save into ``train.report``
(metrics = merged log history, checkpoint = the saved HF checkpoint directory).
``prepare_trainer`` lets ``train_dataset`` / ``eval_dataset`` be ray_amd Data shards
(``train.get_dataset_shard``) or any iterable of ready batches.
"""

from __future__ import annotations

import os
import shutil
import tempfile

from ray_amd import train

try:
    import transformers
    from torch.utils.data import DataLoader, Dataset, IterableDataset
    from transformers.trainer_callback import TrainerCallback

    _IMPORT_ERROR = None
except ImportError as e:  # pragma: no cover
    TrainerCallback = object
    _IMPORT_ERROR = e


class RayTrainReportCallback(TrainerCallback):
    CHECKPOINT_NAME = "checkpoint"

    def on_save(self, args, state, control, **kwargs):
        metrics = {}
        for log in state.log_history:
            metrics.update(log)
        src = transformers.trainer_utils.get_last_checkpoint(args.output_dir)
        with tempfile.TemporaryDirectory() as tmp:
            ckpt = None
            if src is not None:
                shutil.copytree(src, os.path.join(tmp, self.CHECKPOINT_NAME))
                ckpt = train.Checkpoint.from_directory(tmp)
            train.report(metrics, checkpoint=ckpt)


class RayTorchIterableDataset(IterableDataset if _IMPORT_ERROR is None else object):
    """Wraps a ray_amd Data shard (or any iterable of batches) for a DataLoader."""

    def __init__(self, data_iterable, batch_size=None):
        super().__init__()
        self.data_iterable = data_iterable
        self.batch_size = batch_size

    def __iter__(self):
        it = self.data_iterable
        if hasattr(it, "iter_torch_batches"):
            it = it.iter_torch_batches(batch_size=self.batch_size or 8)
        return iter(it)


def _is_ray_iterable(ds) -> bool:
    return ds is not None and not isinstance(ds, Dataset) and (
        hasattr(ds, "iter_torch_batches") or hasattr(ds, "__iter__"))


def prepare_trainer(trainer):
    if _IMPORT_ERROR is not None:
        raise _IMPORT_ERROR
    base = trainer.__class__

    class RayTransformersTrainer(base):
        def get_train_dataloader(self):
            if _is_ray_iterable(self.train_dataset):
                ds = RayTorchIterableDataset(self.train_dataset,
                                             self.args.per_device_train_batch_size)
                return DataLoader(ds, batch_size=1, collate_fn=lambda x: x[0])
            return super().get_train_dataloader()

        def get_eval_dataloader(self, eval_dataset=None):
            eval_dataset = self.eval_dataset if eval_dataset is None else eval_dataset
            if _is_ray_iterable(eval_dataset):
                ds = RayTorchIterableDataset(eval_dataset, self.args.per_device_eval_batch_size)
                return DataLoader(ds, batch_size=1, collate_fn=lambda x: x[0])
            return super().get_eval_dataloader(eval_dataset)

    trainer.__class__ = RayTransformersTrainer
    return trainer


__all__ = ["RayTrainReportCallback", "prepare_trainer", "RayTorchIterableDataset"]
