"""``ModelCatalog`` (reference: rllib/models/catalog.py): custom model and action
distribution registries of the old API stack, and the default catalog choices."""

from __future__ import annotations

import numpy as np

from ray_amd.rllib.env import spaces

MODEL_DEFAULTS = {"fcnet_hiddens": [256, 256], "fcnet_activation": "tanh",
                  "conv_filters": None, "conv_activation": "relu", "use_lstm": False,
                  "lstm_cell_size": 256, "max_seq_len": 20, "vf_share_layers": False,
                  "free_log_std": False, "custom_model": None, "custom_model_config": {},
                  "custom_action_dist": None}


class ModelCatalog:
    _custom_models: dict = {}
    _custom_action_dists: dict = {}

    @staticmethod
    def register_custom_model(model_name: str, model_class) -> None:
        ModelCatalog._custom_models[model_name] = model_class

    @staticmethod
    def register_custom_action_dist(action_dist_name: str, action_dist_class) -> None:
        ModelCatalog._custom_action_dists[action_dist_name] = action_dist_class

    @staticmethod
    def get_action_shape(action_space, framework="torch"):
        if isinstance(action_space, spaces.Discrete):
            return np.int64, (None,)
        return np.float32, (None,) + tuple(action_space.shape)

    @staticmethod
    def get_action_dist(action_space, config=None, dist_type=None, framework="torch",
                        **kwargs):
        """(distribution name or class, number of distribution inputs)."""
        config = config or {}
        name = config.get("custom_action_dist")
        if name:
            return ModelCatalog._custom_action_dists[name], config.get("num_outputs")
        if isinstance(action_space, spaces.Discrete):
            return "Categorical", int(action_space.n)
        return "DiagGaussian", 2 * int(np.prod(action_space.shape))

    @staticmethod
    def get_model_v2(obs_space, action_space, num_outputs, model_config, framework="torch",
                     name="default_model", model_interface=None, default_model=None,
                     **model_kwargs):
        """An instance of the registered custom model (or ``default_model``) with the
        old-stack constructor signature."""
        cfg = dict(MODEL_DEFAULTS)
        cfg.update(model_config or {})
        cname = cfg.get("custom_model")
        if cname:
            cls = cname if isinstance(cname, type) else ModelCatalog._custom_models.get(cname)
            if cls is None:
                raise ValueError(f"custom model {cname!r} is not registered "
                                 "(ModelCatalog.register_custom_model)")
            kw = dict(cfg.get("custom_model_config") or {})
            kw.update(model_kwargs)
            return cls(obs_space, action_space, num_outputs, cfg, name, **kw)
        if default_model is not None:
            return default_model(obs_space, action_space, num_outputs, cfg, name)
        from ray_amd.rllib.core.rl_module.default import RLModule

        return RLModule(obs_space, action_space, cfg)

    @staticmethod
    def get_preprocessor_for_space(observation_space, options=None):
        """The old-stack preprocessor of ``observation_space`` (models/preprocessors.py).
        ray_amd's own modules take observations unflattened; this is for old-stack code."""
        from ray_amd.rllib.models.preprocessors import get_preprocessor

        return get_preprocessor(observation_space)(observation_space, options)

    @staticmethod
    def get_preprocessor(env, options=None):
        return ModelCatalog.get_preprocessor_for_space(env.observation_space, options)


def _custom_model_module(cfg: dict, observation_space, action_space):
    """RLModule adapter over a ModelV2 named by ``model["custom_model"]``."""
    import torch

    from ray_amd.rllib.core.rl_module.rl_module import TorchRLModule, ValueFunctionAPI

    mc = dict(MODEL_DEFAULTS)
    mc.update(cfg.get("model") or {})
    _, n_out = ModelCatalog.get_action_dist(action_space, mc)

    class _ModelV2Module(TorchRLModule, ValueFunctionAPI):
        def setup(self):
            self.model = ModelCatalog.get_model_v2(observation_space, action_space, n_out, mc)

        def _forward(self, batch, **kw):
            obs = batch["obs"]
            if not torch.is_floating_point(obs):
                obs = obs.float()
            out, _ = self.model({"obs": obs, "obs_flat": obs.reshape(obs.shape[0], -1)},
                                [], None)
            return {"action_dist_inputs": out, "vf_preds": self.model.value_function()}

        def compute_values(self, batch, embeddings=None):
            return self._forward(batch)["vf_preds"]

    return _ModelV2Module(observation_space, action_space, model_config=mc)


from ray_amd.rllib.models.action_dist import ActionDistribution  # noqa: E402,F401
from ray_amd.rllib.models.modelv2 import ModelV2  # noqa: E402,F401
from ray_amd.rllib.models.preprocessors import Preprocessor  # noqa: E402,F401

__all__ = ["ActionDistribution", "ModelCatalog", "ModelV2", "MODEL_DEFAULTS", "Preprocessor"]
