"""Classic-stack Policy API (reference: rllib/policy/policy.py, torch_policy_v2.py).

``Policy`` is the old-stack unit of "model + action computation + (optionally) loss":
``compute_actions`` / ``compute_single_action``, ``learn_on_batch``, weights and state,
checkpoints. New code uses RLModules and Learners (this framework's default path);
``Policy`` stays for users porting old-stack code, and ``Algorithm.get_policy()``
returns a Policy bound to the trained module.

``TorchPolicy`` wraps a user ``torch.nn.Module`` (observations -> action logits for
Discrete spaces, or means for Box spaces) and an optional ``loss_fn(policy, model,
batch) -> loss``; ``learn_on_batch`` runs one optimizer step on a SampleBatch.
"""

from __future__ import annotations

import os
import pickle

import numpy as np
import torch

from ray_amd.rllib.env import spaces


class Policy:
    def __init__(self, observation_space, action_space, config: dict | None = None):
        self.observation_space = observation_space
        self.action_space = action_space
        self.config = dict(config or {})
        self.global_timestep = 0

    def compute_actions(self, obs_batch, state_batches=None, prev_action_batch=None,
                        prev_reward_batch=None, info_batch=None, episodes=None,
                        explore=None, timestep=None, **kwargs):
        """-> (actions [B, ...], state_outs list, extra fetches dict)."""
        raise NotImplementedError

    def compute_single_action(self, obs=None, state=None, *, prev_action=None,
                              prev_reward=None, info=None, explore=None, timestep=None,
                              **kwargs):
        acts, st, extra = self.compute_actions(
            np.asarray(obs)[None], [np.asarray(s)[None] for s in state] if state else None,
            explore=explore, timestep=timestep, **kwargs)
        return (acts[0], [s[0] for s in st] if st else [],
                {k: v[0] for k, v in extra.items()} if extra else {})

    def learn_on_batch(self, samples) -> dict:
        raise NotImplementedError

    def get_weights(self):
        raise NotImplementedError

    def set_weights(self, weights) -> None:
        raise NotImplementedError

    def get_initial_state(self) -> list:
        return []

    def is_recurrent(self) -> bool:
        return bool(self.get_initial_state())

    def num_state_tensors(self) -> int:
        return len(self.get_initial_state())

    def get_state(self) -> dict:
        return {"weights": self.get_weights(), "global_timestep": self.global_timestep,
                "policy_spec": (type(self), self.observation_space, self.action_space,
                                self.config)}

    def set_state(self, state: dict) -> None:
        self.set_weights(state["weights"])
        self.global_timestep = state.get("global_timestep", 0)

    def on_global_var_update(self, global_vars: dict) -> None:
        self.global_timestep = global_vars.get("timestep", self.global_timestep)

    def export_checkpoint(self, export_dir: str) -> None:
        os.makedirs(export_dir, exist_ok=True)
        with open(os.path.join(export_dir, "policy_state.pkl"), "wb") as f:
            import cloudpickle

            cloudpickle.dump(self.get_state(), f)

    @staticmethod
    def from_checkpoint(checkpoint: str) -> "Policy":
        with open(os.path.join(checkpoint, "policy_state.pkl"), "rb") as f:
            st = pickle.load(f)
        cls, obs, act, cfg = st["policy_spec"]
        p = cls.__new__(cls)
        if hasattr(p, "_from_state"):
            p._from_state(obs, act, cfg, st)
        else:
            Policy.__init__(p, obs, act, cfg)
            p.set_state(st)
        return p


class TorchPolicy(Policy):
    def __init__(self, observation_space, action_space, config: dict | None = None, *,
                 model: torch.nn.Module, loss_fn=None, optimizer=None):
        super().__init__(observation_space, action_space, config)
        self.model = model
        self.loss_fn = loss_fn
        self.device = torch.device(self.config.get("device", "cpu"))
        self.model.to(self.device)
        self.optimizer = optimizer or torch.optim.Adam(self.model.parameters(),
                                                       lr=self.config.get("lr", 1e-3))

    def _from_state(self, obs, act, cfg, st):
        raise TypeError("TorchPolicy checkpoints need the model: construct the policy and "
                        "call set_state(...) with the checkpoint's state instead")

    def _dist(self, out):
        if isinstance(self.action_space, spaces.Discrete):
            return torch.distributions.Categorical(logits=out)
        std = torch.exp(torch.as_tensor(self.config.get("log_std", -0.5), device=out.device))
        return torch.distributions.Normal(out, std)

    def compute_actions(self, obs_batch, state_batches=None, explore=None, **kwargs):
        explore = self.config.get("explore", True) if explore is None else explore
        obs = torch.as_tensor(np.asarray(obs_batch), dtype=torch.float32, device=self.device)
        with torch.no_grad():
            out = self.model(obs)
            if explore:
                d = self._dist(out)
                act = d.sample()
                logp = d.log_prob(act)
                if logp.dim() > 1:
                    logp = logp.sum(-1)
            else:
                act = out.argmax(-1) if isinstance(self.action_space, spaces.Discrete) \
                    else out
                logp = torch.zeros(act.shape[0], device=out.device)
        self.global_timestep += len(obs_batch)
        return (act.cpu().numpy(), [], {"action_logp": logp.cpu().numpy(),
                                       "action_dist_inputs": out.cpu().numpy()})

    def action_log_prob(self, obs, actions):
        out = self.model(obs)
        lp = self._dist(out).log_prob(actions)
        return lp.sum(-1) if lp.dim() > 1 else lp

    def learn_on_batch(self, samples) -> dict:
        if self.loss_fn is None:
            raise NotImplementedError("TorchPolicy(loss_fn=...) is required for "
                                      "learn_on_batch")
        batch = {k: torch.as_tensor(np.asarray(v), device=self.device)
                 for k, v in dict(samples).items()
                 if isinstance(v, (np.ndarray, list)) and np.asarray(v).dtype != object}
        self.model.train()
        loss = self.loss_fn(self, self.model, batch)
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        gc = self.config.get("grad_clip")
        if gc:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), gc)
        self.optimizer.step()
        self.model.eval()
        return {"learner_stats": {"total_loss": float(loss.detach())}}

    def get_weights(self):
        return {k: v.detach().cpu().numpy() for k, v in self.model.state_dict().items()}

    def set_weights(self, weights) -> None:
        self.model.load_state_dict({k: torch.as_tensor(v) for k, v in weights.items()})


__all__ = ["Policy", "TorchPolicy"]


class TFPolicy(Policy):
    """TensorFlow policies (reference: rllib/policy/tf_policy.py) need tensorflow, which
    this framework does not ship: constructing one fails like the reference does without
    it. Torch policies (``TorchPolicy``) are the supported kind."""

    def __init__(self, *args, **kwargs):
        try:
            import tensorflow  # noqa: F401
        except ImportError:
            raise ImportError("TFPolicy requires tensorflow, which is not installed; use "
                              "TorchPolicy") from None
        raise NotImplementedError("TFPolicy: RLlib modules here are torch modules")
