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

    # --------------------------------------------------- reference helper surface
    def compute_actions_from_input_dict(self, input_dict, explore=None, timestep=None,
                                        episodes=None, **kwargs):
        d = dict(input_dict)
        states = [v for k, v in sorted(d.items()) if k.startswith("state_in")]
        return self.compute_actions(d["obs"], states or None,
                                    prev_action_batch=d.get("prev_actions"),
                                    prev_reward_batch=d.get("prev_rewards"),
                                    explore=explore, timestep=timestep, **kwargs)

    def compute_log_likelihoods(self, actions, obs_batch, state_batches=None,
                                prev_action_batch=None, prev_reward_batch=None,
                                actions_normalized: bool = True, in_training: bool = True):
        raise NotImplementedError

    def postprocess_trajectory(self, sample_batch, other_agent_batches=None, episode=None):
        """Per-trajectory postprocessing (GAE and the like); identity by default."""
        return sample_batch

    def loss(self, model, dist_class, train_batch):
        raise NotImplementedError

    def compute_gradients(self, postprocessed_batch):
        raise NotImplementedError

    def apply_gradients(self, gradients) -> None:
        raise NotImplementedError

    # multi-GPU "tower" API: load once, learn on slices
    def load_batch_into_buffer(self, batch, buffer_index: int = 0) -> int:
        self._loaded = getattr(self, "_loaded", {})
        self._loaded[buffer_index] = batch
        return len(batch)

    def get_num_samples_loaded_into_buffer(self, buffer_index: int = 0) -> int:
        b = getattr(self, "_loaded", {}).get(buffer_index)
        return len(b) if b is not None else 0

    def learn_on_loaded_batch(self, offset: int = 0, buffer_index: int = 0):
        b = self._loaded[buffer_index]
        mb = self.config.get("minibatch_size") or self.config.get("sgd_minibatch_size") \
            or len(b)
        sl = b.slice(offset, min(offset + mb, len(b))) if hasattr(b, "slice") else b
        return self.learn_on_batch(sl)

    def learn_on_batch_from_replay_buffer(self, replay_actor, policy_id: str):
        """Sample a train batch from a (local or actor) replay buffer and learn on it."""
        import ray_amd as ray

        n = self.config.get("train_batch_size", 32)
        samp = replay_actor.sample.remote(n) if hasattr(replay_actor.sample, "remote") \
            else replay_actor.sample(n)
        batch = ray.get(samp) if isinstance(samp, ray.ObjectRef) else samp
        if isinstance(batch, dict) and policy_id in batch:
            batch = batch[policy_id]
        if not batch:
            return {}
        from ray_amd.rllib.policy_sample_batch import SampleBatch

        return self.learn_on_batch(SampleBatch({k: v for k, v in dict(batch).items()
                                                if k != "batch_indexes"}))

    def get_exploration_state(self) -> dict:
        e = getattr(self, "exploration", None)
        return e.get_state() if e is not None else {}

    def export_model(self, export_dir: str, onnx=None) -> None:
        os.makedirs(export_dir, exist_ok=True)
        m = getattr(self, "model", None)
        if m is None:
            raise NotImplementedError("this policy has no torch model to export")
        torch.save(m.state_dict(), os.path.join(export_dir, "model.pt"))

    def import_model_from_h5(self, import_file: str) -> None:
        raise NotImplementedError("h5 (Keras) weights need tensorflow")

    def apply(self, func, *args, **kwargs):
        return func(self, *args, **kwargs)

    def get_host(self) -> str:
        import socket

        return socket.gethostname()

    def get_session(self):
        return None

    def init_view_requirements(self) -> None:
        self.view_requirements = {}

    def make_rl_module(self):
        return getattr(self, "model", None)

    def maybe_add_time_dimension(self, input_dict, seq_lens=None, framework="torch"):
        return input_dict

    def maybe_remove_time_dimension(self, input_dict):
        return input_dict

    def get_connector_metrics(self) -> dict:
        return {}

    def reset_connectors(self, env_id) -> None:
        pass

    def restore_connectors(self, state) -> None:
        pass

    @staticmethod
    def from_state(state: dict) -> "Policy":
        cls, obs, act, cfg = state["policy_spec"]
        p = cls.__new__(cls)
        if hasattr(p, "_from_state"):
            p._from_state(obs, act, cfg, state)
        else:
            Policy.__init__(p, obs, act, cfg)
            p.set_state(state)
        return p

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

    def compute_log_likelihoods(self, actions, obs_batch, state_batches=None,
                                prev_action_batch=None, prev_reward_batch=None,
                                actions_normalized: bool = True, in_training: bool = True):
        obs = torch.as_tensor(np.asarray(obs_batch), dtype=torch.float32, device=self.device)
        a = torch.as_tensor(np.asarray(actions), device=self.device)
        with torch.no_grad():
            return self.action_log_prob(obs, a).cpu().numpy()

    def loss(self, model, dist_class, train_batch):
        if self.loss_fn is None:
            raise NotImplementedError("TorchPolicy(loss_fn=...) defines the loss")
        return self.loss_fn(self, model, train_batch)

    def _tensor_batch(self, samples):
        return {k: torch.as_tensor(np.asarray(v), device=self.device)
                for k, v in dict(samples).items()
                if isinstance(v, (np.ndarray, list)) and np.asarray(v).dtype != object}

    def compute_gradients(self, postprocessed_batch):
        """(gradients as numpy arrays in parameter order, info)."""
        self.model.train()
        loss = self.loss(self.model, None, self._tensor_batch(postprocessed_batch))
        self.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        grads = [None if p.grad is None else p.grad.detach().cpu().numpy()
                 for p in self.model.parameters()]
        self.model.eval()
        return grads, {"learner_stats": {"total_loss": float(loss.detach())}}

    def apply_gradients(self, gradients) -> None:
        for p, g in zip(self.model.parameters(), gradients):
            p.grad = None if g is None else torch.as_tensor(g, device=p.device)
        gc = self.config.get("grad_clip")
        if gc:
            torch.nn.utils.clip_grad_norm_(self.model.parameters(), gc)
        self.optimizer.step()

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
