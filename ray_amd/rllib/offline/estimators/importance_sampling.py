"""Importance-sampling estimators (reference: rllib/offline/estimators/
importance_sampling.py:17, weighted_importance_sampling.py).

With p_t = prod_{t' <= t} pi_e(a_t' | s_t') / pi_b(a_t' | s_t') the cumulative importance
ratio of an episode:

* IS:  V = sum_t gamma^t p_t r_t
* WIS: V = sum_t gamma^t (p_t / w_t) r_t, with w_t the mean of p_t over the episodes of
  the batch that reach step t (step-wise weighted IS)

Single-step samples (bandits, ``split_batch_by_episode=False``): IS uses the per-row
ratio w = pi_e / pi_b times r; WIS divides by the batch mean of w.
"""

from __future__ import annotations

import numpy as np

from .off_policy_estimator import OffPolicyEstimator


def cumulative_ratios(new_prob, old_prob) -> np.ndarray:
    return np.cumprod(np.asarray(new_prob, np.float64) / np.asarray(old_prob, np.float64))


class ImportanceSampling(OffPolicyEstimator):
    def estimate_on_single_episode(self, episode) -> dict:
        r = np.asarray(episode["rewards"], np.float64)
        p = cumulative_ratios(self.compute_action_probs(episode), episode["action_prob"])
        disc = self.gamma ** np.arange(len(r))
        return {"v_behavior": float((disc * r).sum()), "v_target": float((disc * p * r).sum())}

    def estimate_on_single_step_samples(self, batch) -> dict:
        r = np.asarray(batch["rewards"], np.float64)
        w = self.compute_action_probs(batch) / np.asarray(batch["action_prob"], np.float64)
        return {"v_behavior": r, "v_target": w * r}


class WeightedImportanceSampling(OffPolicyEstimator):
    def on_before_split_batch_by_episode(self, batch):
        self._sum_p, self._count, self._p = [], [], {}
        return batch

    def peek_on_single_episode(self, episode) -> None:
        p = cumulative_ratios(self.compute_action_probs(episode), episode["action_prob"])
        for t, pt in enumerate(p):
            if t >= len(self._sum_p):
                self._sum_p.append(pt)
                self._count.append(1.0)
            else:
                self._sum_p[t] += pt
                self._count[t] += 1.0
        key = int(np.asarray(episode["eps_id"])[0]) if "eps_id" in episode else id(episode)
        if key in self._p:
            raise ValueError(f"episode {key} appears twice in the batch")
        self._p[key] = p

    def estimate_on_single_episode(self, episode) -> dict:
        key = int(np.asarray(episode["eps_id"])[0]) if "eps_id" in episode else id(episode)
        p = self._p[key]
        r = np.asarray(episode["rewards"], np.float64)
        w = np.asarray(self._sum_p[:len(r)]) / np.asarray(self._count[:len(r)])
        disc = self.gamma ** np.arange(len(r))
        return {"v_behavior": float((disc * r).sum()),
                "v_target": float((disc * (p / w) * r).sum())}

    def estimate_on_single_step_samples(self, batch) -> dict:
        r = np.asarray(batch["rewards"], np.float64)
        w = self.compute_action_probs(batch) / np.asarray(batch["action_prob"], np.float64)
        return {"v_behavior": r, "v_target": w * r / w.mean()}
