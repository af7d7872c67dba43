"""Ray Train torch integration (reference: python/ray/train/torch/__init__.py)."""

from __future__ import annotations

import os
import tempfile

import torch

from ray_amd.train._checkpoint import Checkpoint
from ray_amd.train.data_parallel_trainer import DataParallelTrainer
from ray_amd.train.torch.config import TorchConfig
from ray_amd.train.torch.train_loop_utils import (accelerate, backward, enable_reproducibility,
                                                  get_device, get_devices, prepare_data_loader,
                                                  prepare_model, prepare_optimizer)


class TorchTrainer(DataParallelTrainer):
    """Data-parallel PyTorch training on one actor per GPU (RCCL over xGMI)."""

    _default_backend_config = TorchConfig

    def __init__(self, train_loop_per_worker, *, train_loop_config=None, torch_config=None,
                 scaling_config=None, run_config=None, datasets=None, dataset_config=None,
                 resume_from_checkpoint=None, metadata=None):
        super().__init__(train_loop_per_worker, train_loop_config=train_loop_config,
                         backend_config=torch_config or TorchConfig(),
                         scaling_config=scaling_config, run_config=run_config,
                         datasets=datasets, dataset_config=dataset_config,
                         resume_from_checkpoint=resume_from_checkpoint, metadata=metadata)


class TorchCheckpoint(Checkpoint):
    MODEL_FILENAME = "model.pt"

    @classmethod
    def from_state_dict(cls, state_dict, *, preprocessor=None):
        d = tempfile.mkdtemp(prefix="ra_torch_ckpt_")
        torch.save(state_dict, os.path.join(d, cls.MODEL_FILENAME))
        c = cls(d)
        if preprocessor is not None:
            c.set_preprocessor(preprocessor)
        return c

    @classmethod
    def from_model(cls, model, *, preprocessor=None):
        d = tempfile.mkdtemp(prefix="ra_torch_ckpt_")
        torch.save(model, os.path.join(d, cls.MODEL_FILENAME))
        c = cls(d)
        if preprocessor is not None:
            c.set_preprocessor(preprocessor)
        return c

    def get_model(self, model=None):
        obj = torch.load(os.path.join(self._local_path(), self.MODEL_FILENAME),
                         weights_only=False)
        if isinstance(obj, dict) and model is not None:
            model.load_state_dict(obj)
            return model
        return obj


from ray_amd.train.torch.torch_predictor import (TorchDetectionPredictor,  # noqa: E402
                                                  TorchPredictor)

__all__ = ["TorchTrainer", "TorchConfig", "TorchCheckpoint", "TorchPredictor",
           "TorchDetectionPredictor", "prepare_model",
           "prepare_data_loader", "prepare_optimizer", "get_device", "get_devices", "backward",
           "enable_reproducibility", "accelerate"]
