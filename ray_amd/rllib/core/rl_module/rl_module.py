"""The RLModule extensibility layer (reference: rllib/core/rl_module/rl_module.py:58
(RLModuleSpec), rllib/core/rl_module/torch/torch_rl_module.py, rllib/core/rl_module/apis/
value_function_api.py, rllib/core/models/torch/encoder.py:294 (TorchLSTMEncoder)).

* ``RLModuleSpec`` / ``MultiRLModuleSpec`` describe a module (class, spaces, model config);
  ``AlgorithmConfig.rl_module(rl_module_spec=...)`` hands one to every Learner and
  EnvRunner, which build it with ``build_module``.
* ``TorchRLModule`` is the base for user modules: ``setup()`` builds the layers,
  ``_forward_inference / _forward_exploration / _forward_train`` map a batch dict
  (``Columns.OBS`` ...) to outputs (``Columns.ACTION_DIST_INPUTS``, optionally
  ``Columns.VF_PREDS``); value-based algorithms also need ``compute_values`` (the
  ValueFunctionAPI). Stateful modules return ``get_initial_state()`` and read / write
  ``Columns.STATE_IN`` / ``Columns.STATE_OUT``.
* Without a spec the built-in MI355X modules run (``default.RLModule``: HIP conv encoder,
  fused PPO heads+loss kernel, learner HIP graphs); ``model_config["use_lstm"]`` selects
  ``LSTMActorCritic``, the stateful default.

Internally Learners and EnvRunners talk to every module through one small interface
(``forward_inference(obs)``, ``forward_train(obs, idx)``, ``value(obs)``,
``sample_actions(dist_inputs, explore)``); ``_UserModuleAdapter`` provides it for user
modules.
"""

from __future__ import annotations

import dataclasses

import numpy as np
import torch
import torch.nn as nn

from ray_amd.rllib.core.rl_module.checkpoint import (CheckpointableModuleMixin,  # noqa: F401
                                                  MultiRLModule)

from ray_amd.rllib.core.columns import Columns
from ray_amd.rllib.core.rl_module import default as D
from ray_amd.rllib.env import spaces


class ValueFunctionAPI:
    """Marker + contract: ``compute_values(batch, embeddings=None) -> [B]`` values."""

    def compute_values(self, batch, embeddings=None):
        raise NotImplementedError


class TorchRLModule(CheckpointableModuleMixin, nn.Module):
    """Base class of user RLModules (reference: TorchRLModule / RLModule new API)."""

    framework = "torch"

    def __init__(self, observation_space=None, action_space=None, inference_only=False,
                 model_config=None, catalog_class=None, **kwargs):
        nn.Module.__init__(self)
        self.observation_space = observation_space
        self.action_space = action_space
        self.inference_only = inference_only
        self.model_config = dict(model_config or {})
        self.catalog_class = catalog_class
        self.setup()

    def setup(self):
        """Build the module's layers (called from __init__)."""

    # ---- forward passes (override _forward or the three specific ones)
    def _forward(self, batch, **kwargs):
        raise NotImplementedError(f"{type(self).__name__} must implement _forward or the "
                                  "_forward_{inference,exploration,train} methods")

    def _forward_inference(self, batch, **kwargs):
        return self._forward(batch, **kwargs)

    def _forward_exploration(self, batch, **kwargs):
        return self._forward(batch, **kwargs)

    def _forward_train(self, batch, **kwargs):
        return self._forward(batch, **kwargs)

    def forward_inference(self, batch, **kwargs):
        return self._forward_inference(batch, **kwargs)

    def forward_exploration(self, batch, **kwargs):
        return self._forward_exploration(batch, **kwargs)

    def forward_train(self, batch, **kwargs):
        return self._forward_train(batch, **kwargs)

    # ---- state
    def get_initial_state(self) -> dict:
        return {}

    def is_stateful(self) -> bool:
        return bool(self.get_initial_state())

    def get_state(self, *a, **k):
        return {k_: v.detach().cpu() for k_, v in self.state_dict().items()}

    def set_state(self, state):
        self.load_state_dict(state)

    def _ctor_args(self):
        return ((self.observation_space, self.action_space),
                {"inference_only": self.inference_only, "model_config": self.model_config,
                 "catalog_class": self.catalog_class})


@dataclasses.dataclass
class RLModuleSpec:
    """How to build one RLModule (reference: rl_module.py:58)."""

    module_class: type | None = None
    observation_space: object = None
    action_space: object = None
    inference_only: bool = False
    model_config: dict | None = None
    catalog_class: object = None
    load_state_path: str | None = None

    def build(self):
        if self.module_class is None:
            raise ValueError("RLModuleSpec.module_class is not set")
        return self.module_class(observation_space=self.observation_space,
                                 action_space=self.action_space,
                                 inference_only=self.inference_only,
                                 model_config=dict(self.model_config or {}),
                                 catalog_class=self.catalog_class)

    def update(self, other, override=True):
        for f in dataclasses.fields(self):
            v = getattr(other, f.name)
            if v is not None and (override or getattr(self, f.name) is None):
                setattr(self, f.name, v)
        return self


@dataclasses.dataclass
class MultiRLModuleSpec:
    """One RLModuleSpec per module id (reference: multi_rl_module.py)."""

    rl_module_specs: dict = dataclasses.field(default_factory=dict)

    def __getitem__(self, mid):
        return self.rl_module_specs[mid]

    def build(self):
        return {mid: s.build() for mid, s in self.rl_module_specs.items()}


def _discrete(action_space):
    return isinstance(action_space, spaces.Discrete) or hasattr(action_space, "n")


class _SamplingMixin:
    def sample_actions(self, dist_inputs, explore=True):
        return D.RLModule.sample_actions(self, dist_inputs, explore)


class _UserModuleAdapter(_SamplingMixin, nn.Module):
    """The Learner / EnvRunner interface over a user TorchRLModule (the user module is the
    submodule ``m``; parameters, weights and checkpoints are the user module's)."""

    is_image = False
    vf_encoder = None

    def __init__(self, module: TorchRLModule):
        super().__init__()
        self.m = module
        self.discrete = _discrete(module.action_space)
        if not self.discrete:
            self.act_dim = int(np.prod(module.action_space.shape))

    def is_stateful(self):
        return self.m.is_stateful()

    def get_initial_state(self):
        return self.m.get_initial_state()

    def _out(self, out, batch, want_values):
        if want_values and Columns.VF_PREDS not in out:
            if not isinstance(self.m, ValueFunctionAPI) and \
                    type(self.m).compute_values is ValueFunctionAPI.compute_values:
                raise NotImplementedError(f"{type(self.m).__name__} must return "
                                          f"{Columns.VF_PREDS} or implement compute_values")
            out = dict(out)
            out[Columns.VF_PREDS] = self.m.compute_values(batch, out.get(Columns.EMBEDDINGS))
        return out

    def forward_inference(self, obs, state=None):
        b = {Columns.OBS: obs}
        if state is not None:
            b[Columns.STATE_IN] = state
        return self.m.forward_inference(b)

    def forward_exploration(self, obs, state=None):
        b = {Columns.OBS: obs}
        if state is not None:
            b[Columns.STATE_IN] = state
        return self.m.forward_exploration(b)

    def forward_train(self, obs, idx=None, **kw):
        if idx is not None:
            obs = obs.index_select(0, idx)
        b = {Columns.OBS: obs, **kw}
        return self._out(self.m.forward_train(b), b, True)

    def value(self, obs):
        b = {Columns.OBS: obs}
        if hasattr(self.m, "compute_values"):
            try:
                return self.m.compute_values(b)
            except NotImplementedError:
                pass
        return self.m.forward_train(b)[Columns.VF_PREDS]


class LSTMActorCritic(_SamplingMixin, nn.Module):
    """Stateful default actor-critic: MLP encoder -> LSTM cell -> policy / value heads
    (reference: TorchLSTMEncoder, rllib/core/models/torch/encoder.py:294; model_config
    ``use_lstm``, ``lstm_cell_size``). Time-major training over [T, B] rollout fragments:
    the state starts at each fragment's recorded ``state_in`` and is zeroed where an
    episode begins inside the fragment (``resets``)."""

    is_image = False
    vf_encoder = None

    def __init__(self, observation_space, action_space, model_config=None):
        super().__init__()
        cfg = dict(model_config or {})
        self.discrete = _discrete(action_space)
        d = int(np.prod(observation_space.shape))
        self.encoder = D.MLP(d, cfg.get("fcnet_hiddens", [64]),
                             cfg.get("fcnet_activation", "tanh"))
        self.cell_size = int(cfg.get("lstm_cell_size", 64))
        self.lstm = nn.LSTMCell(self.encoder.out_dim, self.cell_size)
        if self.discrete:
            n_out = action_space.n
        else:
            self.act_dim = int(np.prod(action_space.shape))
            n_out = 2 * self.act_dim
        self.pi = nn.Linear(self.cell_size, n_out)
        self.vf = nn.Linear(self.cell_size, 1)
        nn.init.orthogonal_(self.pi.weight, 0.01)
        nn.init.zeros_(self.pi.bias)

    def is_stateful(self):
        return True

    def get_initial_state(self):
        z = np.zeros(self.cell_size, np.float32)
        return {"h": z, "c": z.copy()}

    def step(self, obs, state):
        """One time step for a batch: obs [B, ...], state {"h","c"} [B, H] -> (logits,
        values, new state)."""
        x = self.encoder(obs.reshape(obs.shape[0], -1).float())
        h, c = self.lstm(x, (state["h"].float(), state["c"].float()))
        return self.pi(h), self.vf(h).squeeze(-1), {"h": h, "c": c}

    def forward_inference(self, obs, state=None):
        if state is None:
            B = obs.shape[0]
            state = {k: torch.zeros(B, self.cell_size, device=obs.device) for k in ("h", "c")}
        logits, _, st = self.step(obs, state)
        return {Columns.ACTION_DIST_INPUTS: logits, Columns.STATE_OUT: st}

    forward_exploration = forward_inference

    def forward_sequence(self, obs, h0, c0, resets):
        """obs [T, B, ...], h0/c0 [B, H], resets [T, B] (1 where an episode starts at t)
        -> logits [T, B, A], values [T, B], final (h, c)."""
        T, B = obs.shape[:2]
        x = self.encoder(obs.reshape(T * B, -1).float()).view(T, B, -1)
        h, c = h0.float(), c0.float()
        hs = []
        for t in range(T):
            keep = (1.0 - resets[t].float())[:, None]
            h, c = self.lstm(x[t], (h * keep, c * keep))
            hs.append(h)
        H = torch.stack(hs)
        return self.pi(H), self.vf(H).squeeze(-1), (h, c)


def build_module(cfg: dict, observation_space, action_space, module_id=None):
    """The module a Learner / EnvRunner runs for ``cfg`` (the algorithm's config dict):
    a user module from ``cfg["_rl_module_spec"]`` (an RLModuleSpec, or a MultiRLModuleSpec
    for multi-agent), the stateful default when ``model["use_lstm"]``, else the built-in
    actor-critic."""
    spec = cfg.get("_rl_module_spec")
    if isinstance(spec, MultiRLModuleSpec):
        spec = spec.rl_module_specs.get(module_id) if module_id is not None else None
    mc = dict(cfg.get("model") or {})
    if spec is not None and spec.module_class is not None:
        s = RLModuleSpec().update(spec)
        s.observation_space = s.observation_space or observation_space
        s.action_space = s.action_space or action_space
        merged = dict(mc)
        merged.update(s.model_config or {})
        s.model_config = merged
        m = s.build()
        if s.load_state_path:
            m.load_state_dict(torch.load(s.load_state_path, weights_only=True))
        if isinstance(m, TorchRLModule):
            return _UserModuleAdapter(m)
        return m
    if mc.get("custom_model"):  # an old-stack ModelV2 (rllib/models ModelCatalog)
        from ray_amd.rllib.models import _custom_model_module

        return _UserModuleAdapter(_custom_model_module(cfg, observation_space, action_space))
    if mc.get("use_lstm"):
        return LSTMActorCritic(observation_space, action_space, mc)
    return D.RLModule(observation_space, action_space, mc)
