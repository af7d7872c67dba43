"""Direct Method and Doubly Robust estimators (reference: rllib/offline/estimators/
direct_method.py, doubly_robust.py:28).

Both fit a Q-model of the target policy on the logged data (FQE by default, or
``q_model_config={"type": cls, ...}``):

* DM: V = V_Q(s_0) = sum_a pi_e(a | s_0) Q(s_0, a) per episode.
* DR: backwards over an episode with V_T = 0,
      V_t = V_Q(s_t) + w_t (r_t + gamma V_{t+1} - Q(s_t, a_t)),  w_t = pi_e / pi_b at t,
  (per-step ratios; with ``normalize_weights`` the ratios are divided by their mean over
  the batch), V = V_0.
"""

from __future__ import annotations

import numpy as np

from .fqe_torch_model import FQETorchModel
from .off_policy_estimator import OffPolicyEstimator


class _QModelEstimator(OffPolicyEstimator):
    def __init__(self, policy, gamma: float, epsilon_greedy: float = 0.0,
                 q_model_config=None):
        super().__init__(policy, gamma, epsilon_greedy)
        cfg = dict(q_model_config or {})
        cls = cfg.pop("type", FQETorchModel)
        cfg["gamma"] = gamma
        self.model = cls(policy=policy, **cfg)
        if not (hasattr(self.model, "estimate_q") and hasattr(self.model, "estimate_v")):
            raise TypeError("the Q-model must implement estimate_q and estimate_v")

    def train(self, batch) -> dict:
        losses = self.model.train(batch)
        return {"loss": float(np.mean(losses)) if len(losses) else float("nan")}


class DirectMethod(_QModelEstimator):
    def estimate_on_single_episode(self, episode) -> dict:
        r = np.asarray(episode["rewards"], np.float64)
        vb = float((self.gamma ** np.arange(len(r)) * r).sum())
        v0 = self.model.estimate_v({k: np.asarray(v)[:1] for k, v in episode.items()})
        return {"v_behavior": vb, "v_target": float(v0[0])}

    def estimate_on_single_step_samples(self, batch) -> dict:
        return {"v_behavior": np.asarray(batch["rewards"], np.float64),
                "v_target": self.model.estimate_v(batch)}


class DoublyRobust(_QModelEstimator):
    def __init__(self, policy, gamma: float, epsilon_greedy: float = 0.0,
                 normalize_weights: bool = True, q_model_config=None):
        super().__init__(policy, gamma, epsilon_greedy, q_model_config)
        self.normalize_weights = normalize_weights
        self._w_mean = 1.0

    def on_before_split_batch_by_episode(self, batch):
        if self.normalize_weights:
            w = self.compute_action_probs(batch) / np.asarray(batch["action_prob"], np.float64)
            self._w_mean = float(w.mean()) if len(w) else 1.0
        return batch

    def estimate_on_single_episode(self, episode) -> dict:
        r = np.asarray(episode["rewards"], np.float64)
        w = self.compute_action_probs(episode) / np.asarray(episode["action_prob"], np.float64)
        w = w / self._w_mean
        q = self.model.estimate_q(episode)
        v = self.model.estimate_v(episode)
        vb = vt = 0.0
        for t in range(len(r) - 1, -1, -1):
            vb = r[t] + self.gamma * vb
            vt = v[t] + w[t] * (r[t] + self.gamma * vt - q[t])
        return {"v_behavior": float(vb), "v_target": float(vt)}

    def estimate_on_single_step_samples(self, batch) -> dict:
        r = np.asarray(batch["rewards"], np.float64)
        w = self.compute_action_probs(batch) / np.asarray(batch["action_prob"], np.float64)
        if self.normalize_weights:
            w = w / w.mean()
        q = self.model.estimate_q(batch)
        v = self.model.estimate_v(batch)
        return {"v_behavior": r, "v_target": v + w * (r - q)}
