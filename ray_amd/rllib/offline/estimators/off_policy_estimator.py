"""Off-policy estimation base classes (reference: rllib/offline/offline_evaluator.py:16,
rllib/offline/estimators/off_policy_estimator.py).

An estimator evaluates a TARGET policy on data logged by a BEHAVIOUR policy. The data is
a batch of transition rows (``obs``, ``actions``, ``rewards``, ``action_prob`` = the
behaviour policy's probability of the logged action, ``eps_id``, ``t``) — the rows
``ray_amd.rllib.offline.read_offline_dataset`` produces — or a ray_amd.data Dataset of
them (``estimate_on_dataset``).

``estimate(batch)`` splits the rows into episodes, lets every episode ``peek`` (for
dataset-wide normalisers such as WIS's), estimates each episode and reports the
reference's metrics: v_behavior (mean discounted return of the logged episodes),
v_target (the estimate for the target policy), their standard deviations, v_gain =
v_target / max(v_behavior, 1e-8) and v_delta = v_target - v_behavior.

The target policy can be an Algorithm's policy view (``algo.get_policy()``), any object
with ``compute_log_likelihoods(actions, obs_batch)``, an RLModule, or a plain callable
``obs -> action probabilities [N, A]`` (discrete actions).
"""

from __future__ import annotations

import numpy as np


class OfflineEvaluator:
    """Interface of offline evaluation (reference: offline_evaluator.py:16)."""

    def __init__(self, policy, **kwargs):
        self.policy = policy

    def estimate(self, batch, **kwargs) -> dict:
        raise NotImplementedError

    def train(self, batch) -> dict:
        """Fit any model the estimate needs (DM / DR: the FQE Q-model)."""
        return {}

    def estimate_on_dataset(self, dataset, *, n_parallelism: int = 1) -> dict:
        """Estimate over a ray_amd.data Dataset of transition rows: the rows are pulled
        through the Data executor (one streaming pass) and estimated episode-wise."""
        cols = {}
        for b in dataset.iter_batches(batch_size=65536):
            for k, v in b.items():
                cols.setdefault(k, []).append(np.asarray(v))
        batch = {k: np.concatenate(v) for k, v in cols.items()}
        self.train(batch)
        return self.estimate(batch)


def split_by_episode(batch: dict) -> list:
    """Rows -> one dict per episode (ordered by ``t`` when present; rows without
    ``eps_id`` are one episode each — the single-step / bandit case)."""
    n = len(batch["rewards"])
    if "eps_id" not in batch:
        return [{k: np.asarray(v)[i:i + 1] for k, v in batch.items()} for i in range(n)]
    eid = np.asarray(batch["eps_id"])
    order = np.lexsort((np.asarray(batch["t"]), eid)) if "t" in batch else \
        np.argsort(eid, kind="stable")
    eid_s = eid[order]
    cuts = np.nonzero(np.diff(eid_s))[0] + 1
    out = []
    for idx in np.split(order, cuts):
        out.append({k: np.asarray(v)[idx] for k, v in batch.items()})
    return out


def _log_likelihoods(policy, obs, actions):
    """log pi(a | s) of the target policy for rows (obs, actions)."""
    import torch

    if hasattr(policy, "compute_log_likelihoods"):
        return np.asarray(policy.compute_log_likelihoods(actions, obs), np.float64)
    if isinstance(policy, torch.nn.Module):
        with torch.no_grad():
            x = torch.as_tensor(np.asarray(obs, np.float32))
            di = policy.forward_inference(x)["action_dist_inputs"].float()
            a = torch.as_tensor(np.asarray(actions))
            if getattr(policy, "discrete", True) and a.dtype in (torch.int64, torch.int32):
                lp = torch.log_softmax(di, -1).gather(-1, a.long()[:, None])[:, 0]
            else:
                from ray_amd.rllib.core.rl_module.default import gaussian_logp

                mean, log_std = di.chunk(2, -1)
                lp = gaussian_logp(a.float(), mean, log_std)
        return lp.double().numpy()
    if callable(policy):
        p = np.asarray(policy(np.asarray(obs)), np.float64)
        a = np.asarray(actions).astype(np.int64)
        return np.log(np.maximum(p[np.arange(len(a)), a], 1e-300))
    raise TypeError(f"cannot compute action likelihoods with a {type(policy).__name__}")


def action_probabilities(policy, obs, n_actions: int) -> np.ndarray:
    """pi(. | s) for every discrete action: [N, A] (used by DM / DR for V = sum pi Q)."""
    obs = np.asarray(obs)
    n = len(obs)
    cols = [np.exp(_log_likelihoods(policy, obs, np.full(n, a, np.int64)))
            for a in range(n_actions)]
    return np.stack(cols, 1)


class OffPolicyEstimator(OfflineEvaluator):
    """reference: rllib/offline/estimators/off_policy_estimator.py."""

    def __init__(self, policy, gamma: float = 0.0, epsilon_greedy: float = 0.0):
        super().__init__(policy)
        self.gamma = float(gamma)
        self.epsilon_greedy = float(epsilon_greedy)

    # hooks (reference names)
    def on_before_split_batch_by_episode(self, batch):
        return batch

    def on_after_split_batch_by_episode(self, episodes):
        return episodes

    def peek_on_single_episode(self, episode) -> None:
        pass

    def estimate_on_single_episode(self, episode) -> dict:
        raise NotImplementedError

    def estimate_on_single_step_samples(self, batch) -> dict:
        raise NotImplementedError

    def compute_action_probs(self, batch) -> np.ndarray:
        p = np.exp(_log_likelihoods(self.policy, batch["obs"], batch["actions"]))
        if self.epsilon_greedy > 0.0:
            n = self._n_actions()
            if n is None:
                raise ValueError("epsilon_greedy needs a discrete action space")
            p = p * (1.0 - self.epsilon_greedy) + self.epsilon_greedy / n
        return p

    def _n_actions(self):
        sp = getattr(self.policy, "action_space", None)
        return getattr(sp, "n", None)

    @staticmethod
    def check_action_prob_in_batch(batch) -> None:
        if "action_prob" not in batch:
            raise ValueError("off-policy estimation needs the behaviour policy's "
                             "'action_prob' per row (recorded from action_logp)")

    def estimate(self, batch, split_batch_by_episode: bool = True) -> dict:
        self.check_action_prob_in_batch(batch)
        if split_batch_by_episode:
            batch = self.on_before_split_batch_by_episode(batch)
            eps = self.on_after_split_batch_by_episode(split_by_episode(batch))
            for ep in eps:
                self.peek_on_single_episode(ep)
            per = [self.estimate_on_single_episode(ep) for ep in eps]
            vb = np.array([p["v_behavior"] for p in per], np.float64)
            vt = np.array([p["v_target"] for p in per], np.float64)
        else:
            per = self.estimate_on_single_step_samples(batch)
            vb = np.asarray(per["v_behavior"], np.float64)
            vt = np.asarray(per["v_target"], np.float64)
        est = {"v_behavior": float(vb.mean()), "v_behavior_std": float(vb.std()),
               "v_target": float(vt.mean()), "v_target_std": float(vt.std())}
        est["v_gain"] = est["v_target"] / max(est["v_behavior"], 1e-8)
        est["v_delta"] = est["v_target"] - est["v_behavior"]
        return est
