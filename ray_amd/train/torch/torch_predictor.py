"""Torch predictors (reference: python/ray/train/torch/torch_predictor.py,
torch_detection_predictor.py).

``TorchPredictor`` runs a ``torch.nn.Module`` in eval mode under ``no_grad`` on one
device: numpy batches become tensors on that device (non-blocking H2D from pinned memory
when the device is a GPU), outputs come back as numpy. ``use_gpu=True`` picks this
process's current HIP device, so a Data actor pool with ``num_gpus=1`` per actor spreads
the models over the node's GPUs. ``amp=True`` runs the forward under bf16 autocast (the
MI355X matrix cores' native input type; outputs are returned as float32).
"""

from __future__ import annotations

import logging

import numpy as np
import torch

from ray_amd.train.predictor import DLPredictor

logger = logging.getLogger(__name__)


def _device(use_gpu: bool) -> torch.device:
    if use_gpu:
        if not torch.cuda.is_available():
            raise RuntimeError("TorchPredictor(use_gpu=True) but no GPU is visible")
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _to_tensor(a, dtype, device):
    t = torch.as_tensor(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    if device.type == "cuda":
        return t.pin_memory().to(device, non_blocking=True)
    return t


class TorchPredictor(DLPredictor):
    def __init__(self, model: torch.nn.Module, preprocessor=None, use_gpu: bool = False,
                 amp: bool = False):
        self.model = model
        self.model.eval()
        self.use_gpu = use_gpu
        self.amp = amp
        self.device = _device(use_gpu)
        self.model.to(self.device)
        super().__init__(preprocessor)

    def __repr__(self):
        return (f"{type(self).__name__}(model={self.model!r}, "
                f"preprocessor={self._preprocessor!r}, use_gpu={self.use_gpu!r})")

    @classmethod
    def from_checkpoint(cls, checkpoint, model: torch.nn.Module | None = None,
                        use_gpu: bool = False, **kwargs) -> "TorchPredictor":
        """``model`` is required when the checkpoint holds a state dict
        (``TorchCheckpoint.from_state_dict``) and ignored for a pickled module."""
        m = checkpoint.get_model(model)
        if isinstance(m, dict):
            raise ValueError("the checkpoint holds a state dict: pass model=<module> to "
                             "load it into")
        return cls(model=m, preprocessor=checkpoint.get_preprocessor(), use_gpu=use_gpu,
                   **kwargs)

    def call_model(self, inputs):
        with torch.no_grad():
            if self.amp and self.device.type == "cuda":
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    return self.model(inputs)
            return self.model(inputs)

    def predict(self, data, dtype=None):
        return super().predict(data, dtype=dtype)

    def _arrays_to_tensors(self, arrays, dtype):
        if isinstance(arrays, dict):
            return {k: _to_tensor(v, dtype[k] if isinstance(dtype, dict) else dtype,
                                  self.device) for k, v in arrays.items()}
        return _to_tensor(arrays, dtype, self.device)

    def _tensor_to_array(self, tensor) -> np.ndarray:
        if not isinstance(tensor, torch.Tensor):
            raise ValueError(
                f"Expected the model to return a torch.Tensor or a dict of them, got "
                f"{type(tensor)}; subclass TorchPredictor and override call_model to map "
                "other outputs")
        t = tensor.detach()
        if t.dtype == torch.bfloat16:
            t = t.float()
        return t.cpu().numpy()


class TorchDetectionPredictor(TorchPredictor):
    """Detection models (torchvision-style): the forward takes a list of CHW image
    tensors and returns one dict per image (``boxes``, ``labels``, ``scores``, ...).
    Output columns are ``pred_<key>``, each an object array holding one array per image
    (images have different numbers of detections)."""

    def _predict_numpy(self, data, dtype=None):
        if isinstance(data, dict):
            if len(data) != 1:
                raise ValueError(
                    f"Expected a single image column, got columns {list(data)}")
            images = next(iter(data.values()))
        else:
            images = data
        inputs = [_to_tensor(img, dtype, self.device) for img in images]
        outputs = self.call_model(inputs)
        if not isinstance(outputs, (list, tuple)) or \
                not all(isinstance(o, dict) for o in outputs):
            raise ValueError("a detection model must return one dict of tensors per image")
        keys = list(outputs[0]) if outputs else ["boxes", "labels", "scores"]
        res = {}
        for k in keys:
            col = np.empty(len(outputs), dtype=object)
            for i, o in enumerate(outputs):
                col[i] = self._tensor_to_array(o[k])
            res["pred_" + k] = col
        return res


__all__ = ["TorchPredictor", "TorchDetectionPredictor"]
