"""Checkpoint API of RLModules (reference: rllib/core/rl_module/rl_module.py
``save_to_path`` / ``from_checkpoint`` / ``save_state`` / ``load_state``, and
multi_rl_module.py ``MultiRLModule``).

A module checkpoint directory holds ``module_state.pt`` (the state dict, read back with
``torch.load(weights_only=True)``) and ``class_and_ctor_args.pkl`` (the module class and
its constructor arguments, written by this framework with cloudpickle). ``from_checkpoint``
rebuilds the module — on any host, without the algorithm — for inference serving."""

from __future__ import annotations

import os
from typing import Dict, Optional

import torch
import torch.nn as nn

STATE_FILE = "module_state.pt"
CTOR_FILE = "class_and_ctor_args.pkl"


class CheckpointableModuleMixin:
    def _ctor_args(self) -> tuple:
        """(args, kwargs) that rebuild this module's structure."""
        return ((self.observation_space, self.action_space),
                {"model_config": getattr(self, "model_config", None)})

    def save_state(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        torch.save({k: v.detach().cpu() for k, v in self.state_dict().items()},
                   os.path.join(path, STATE_FILE))

    def load_state(self, path: str) -> None:
        sd = torch.load(os.path.join(path, STATE_FILE), weights_only=True, map_location="cpu")
        self.load_state_dict(sd)

    def save_to_checkpoint(self, checkpoint_dir_path: str) -> str:
        import cloudpickle

        os.makedirs(checkpoint_dir_path, exist_ok=True)
        self.save_state(checkpoint_dir_path)
        args, kwargs = self._ctor_args()
        with open(os.path.join(checkpoint_dir_path, CTOR_FILE), "wb") as f:
            f.write(cloudpickle.dumps((type(self), args, kwargs)))
        return checkpoint_dir_path

    save_to_path = save_to_checkpoint

    @classmethod
    def from_checkpoint(cls, checkpoint_dir_path: str):
        import cloudpickle

        ctor = os.path.join(checkpoint_dir_path, CTOR_FILE)
        if os.path.exists(ctor):
            with open(ctor, "rb") as f:  # written by save_to_checkpoint above
                klass, args, kwargs = cloudpickle.loads(f.read())
        else:
            raise FileNotFoundError(f"{ctor} not found: not a module checkpoint")
        if os.path.isdir(os.path.join(checkpoint_dir_path, "modules")) and \
                issubclass(klass, MultiRLModule):
            return MultiRLModule.from_checkpoint_dir(checkpoint_dir_path)
        m = klass(*args, **kwargs)
        m.load_state(checkpoint_dir_path)
        return m

    from_path = from_checkpoint

    def as_multi_agent(self, module_id: str = "default_policy") -> "MultiRLModule":
        return MultiRLModule({module_id: self})

    def unwrapped(self):
        return self

    # action-distribution classes (old-stack classes double as the new stack's)
    def _dist_cls(self):
        from ray_amd.rllib.env import spaces
        from ray_amd.rllib.models.action_dist import TorchCategorical, TorchDiagGaussian

        return TorchCategorical if isinstance(self.action_space, spaces.Discrete) \
            else TorchDiagGaussian

    def get_inference_action_dist_cls(self):
        return self._dist_cls()

    def get_exploration_action_dist_cls(self):
        return self._dist_cls()

    def get_train_action_dist_cls(self):
        return self._dist_cls()


class MultiRLModule(nn.ModuleDict):
    """Modules by module id (reference: MultiRLModule): forward passes take and return
    ``{module_id: batch}``; each module checkpoints under ``modules/<id>``."""

    def __init__(self, rl_modules: Optional[Dict[str, nn.Module]] = None, **kw):
        super().__init__(dict(rl_modules or {}))

    def add_module(self, module_id, module=None, *, override: bool = True):  # noqa: D401
        """Add (or with ``override``, replace) the module under ``module_id``. Also the
        torch ``nn.Module.add_module`` that ``ModuleDict.__setitem__`` calls."""
        if not override and module_id in self._modules:
            raise ValueError(f"module {module_id!r} exists (override=True to replace)")
        return nn.Module.add_module(self, str(module_id), module)

    def remove_module(self, module_id, *, raise_err_if_not_found: bool = True):
        if module_id not in self:
            if raise_err_if_not_found:
                raise KeyError(module_id)
            return
        del self[module_id]

    def _run(self, fn, batch, **kw):
        return {mid: getattr(self[mid], fn)(b, **kw) for mid, b in batch.items()}

    def forward_inference(self, batch, **kw):
        return self._run("forward_inference", batch, **kw)

    def forward_exploration(self, batch, **kw):
        return self._run("forward_exploration", batch, **kw)

    def forward_train(self, batch, **kw):
        return self._run("forward_train", batch, **kw)

    def get_state(self, module_ids=None, **kw):
        ids = module_ids or list(self.keys())
        return {mid: {k: v.detach().cpu() for k, v in self[mid].state_dict().items()}
                for mid in ids}

    def set_state(self, state: dict) -> None:
        for mid, sd in state.items():
            if mid in self:
                self[mid].load_state_dict(sd)

    def save_to_checkpoint(self, checkpoint_dir_path: str) -> str:
        import cloudpickle

        os.makedirs(os.path.join(checkpoint_dir_path, "modules"), exist_ok=True)
        for mid, m in self.items():
            m.save_to_checkpoint(os.path.join(checkpoint_dir_path, "modules", str(mid)))
        with open(os.path.join(checkpoint_dir_path, CTOR_FILE), "wb") as f:
            f.write(cloudpickle.dumps((MultiRLModule, (), {"ids": list(self.keys())})))
        return checkpoint_dir_path

    save_to_path = save_to_checkpoint

    @staticmethod
    def from_checkpoint_dir(checkpoint_dir_path: str) -> "MultiRLModule":
        d = os.path.join(checkpoint_dir_path, "modules")
        mods = {}
        for mid in sorted(os.listdir(d)):
            mods[mid] = CheckpointableModuleMixin.from_checkpoint(os.path.join(d, mid))
        return MultiRLModule(mods)

    @classmethod
    def from_checkpoint(cls, checkpoint_dir_path: str) -> "MultiRLModule":
        return cls.from_checkpoint_dir(checkpoint_dir_path)

    def as_multi_agent(self):
        return self

    def unwrapped(self):
        return self
