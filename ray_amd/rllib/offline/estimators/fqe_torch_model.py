"""Fitted-Q Evaluation model for the DM / DR estimators (reference: rllib/offline/
estimators/fqe_torch_model.py).

Learns Q^{pi_e} of the TARGET policy from logged transitions by repeated regression onto
the bootstrapped target  r + gamma * (1 - done) * sum_a' pi_e(a' | s') Q_target(s', a')
(discrete actions), with a Polyak-averaged target network. ``estimate_q`` returns
Q(s_t, a_t) of logged rows and ``estimate_v`` returns V(s_t) = sum_a pi_e(a | s_t) Q(s_t, a).
Runs on the learner device given by ``device`` (the MI355X when one is visible)."""

from __future__ import annotations

import numpy as np
import torch

from .off_policy_estimator import action_probabilities


class FQETorchModel:
    def __init__(self, policy, gamma: float, *, n_actions: int | None = None,
                 model_config=None, n_iters: int = 1, lr: float = 1e-3,
                 min_loss_threshold: float = 1e-4, minibatch_size: int | None = None,
                 tau: float = 1.0, device=None, seed: int = 0, **kw):
        self.policy = policy
        self.gamma = float(gamma)
        sp = getattr(policy, "action_space", None)
        self.n_actions = n_actions or getattr(sp, "n", None)
        if self.n_actions is None:
            raise ValueError("FQE needs a discrete action space (pass n_actions)")
        self.hiddens = list((model_config or {}).get("fcnet_hiddens", [32, 32]))
        self.n_iters, self.lr, self.tau = int(n_iters), float(lr), float(tau)
        self.min_loss = float(min_loss_threshold)
        self.minibatch_size = minibatch_size
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.seed = seed
        self.q = None

    def _build(self, obs_dim):
        g = torch.Generator().manual_seed(self.seed)
        layers, d = [], obs_dim
        for h in self.hiddens:
            lin = torch.nn.Linear(d, h)
            torch.nn.init.orthogonal_(lin.weight, generator=g)
            layers += [lin, torch.nn.ReLU()]
            d = h
        layers.append(torch.nn.Linear(d, self.n_actions))
        self.q = torch.nn.Sequential(*layers).to(self.device)
        self.target = torch.nn.Sequential(*[type(m)(m.in_features, m.out_features)
                                            if isinstance(m, torch.nn.Linear) else
                                            torch.nn.ReLU() for m in layers]).to(self.device)
        self.target.load_state_dict(self.q.state_dict())
        self.opt = torch.optim.Adam(self.q.parameters(), lr=self.lr)

    def _t(self, x, dtype=torch.float32):
        return torch.as_tensor(np.asarray(x), dtype=dtype, device=self.device)

    def train(self, batch) -> list:
        """n_iters passes of FQE regression over the rows; returns the losses."""
        obs = np.asarray(batch["obs"], np.float32).reshape(len(batch["rewards"]), -1)
        if self.q is None:
            self._build(obs.shape[1])
        nobs = np.asarray(batch["next_obs"], np.float32).reshape(obs.shape)
        done = np.asarray(batch["terminateds"], np.float32)
        pi_next = action_probabilities(self.policy, batch["next_obs"], self.n_actions)
        o, no = self._t(obs), self._t(nobs)
        a = self._t(batch["actions"], torch.int64)
        r, d, pn = self._t(batch["rewards"]), self._t(done), self._t(pi_next)
        n = len(r)
        mb = self.minibatch_size or n
        losses = []
        for _ in range(self.n_iters):
            perm = torch.randperm(n, device=self.device)
            for s in range(0, n, mb):
                idx = perm[s:s + mb]
                with torch.no_grad():
                    v_next = (self.target(no[idx]) * pn[idx]).sum(-1)
                    tgt = r[idx] + self.gamma * (1.0 - d[idx]) * v_next
                qa = self.q(o[idx]).gather(-1, a[idx][:, None])[:, 0]
                loss = torch.nn.functional.mse_loss(qa, tgt)
                self.opt.zero_grad()
                loss.backward()
                self.opt.step()
                losses.append(float(loss.detach()))
            with torch.no_grad():  # Polyak update of the target network
                for pt, pq in zip(self.target.parameters(), self.q.parameters()):
                    pt.mul_(1.0 - self.tau).add_(pq, alpha=self.tau)
            if losses and losses[-1] < self.min_loss:
                break
        return losses

    def estimate_q(self, batch) -> np.ndarray:
        obs = np.asarray(batch["obs"], np.float32).reshape(len(batch["actions"]), -1)
        with torch.no_grad():
            q = self.q(self._t(obs)).gather(-1, self._t(batch["actions"], torch.int64)[:, None])
        return q[:, 0].double().cpu().numpy()

    def estimate_v(self, batch) -> np.ndarray:
        obs = np.asarray(batch["obs"], np.float32).reshape(len(batch["obs"]), -1)
        pi = action_probabilities(self.policy, batch["obs"], self.n_actions)
        with torch.no_grad():
            q = self.q(self._t(obs)).double().cpu().numpy()
        return (q * pi).sum(-1)
