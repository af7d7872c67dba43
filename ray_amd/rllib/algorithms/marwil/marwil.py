"""MARWIL and BC (reference: rllib/algorithms/marwil/marwil.py,
torch/marwil_torch_learner.py, rllib/algorithms/bc/bc.py; Wang et al. 2018).

Offline: minibatches come from ``OfflineData`` (recorded experience read through
ray_amd.data — fragment JSON or transition Parquet — with per-episode discounted
returns; ``streaming_split`` shards when there are learner actors). Loss = -E[exp(beta * A / c) * log pi(a|s)] + vf_coeff * 0.5 *
(V(s) - R)^2 with A = R - V(s) and c the running RMS of A (moving-average update
rate ``moving_average_sqd_adv_norm_update_rate``). BC is MARWIL with beta = 0: the
value head is not trained and the loss is plain negative log-likelihood.
An env-runner rollout with the current weights every iteration reports
``episode_return_mean`` (the reference does the same through evaluation)."""

from __future__ import annotations

import numpy as np
import torch

from ray_amd.rllib.algorithms.algorithm import Algorithm
from ray_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_amd.rllib.core.learner import LearnerGroup, TorchLearner
from ray_amd.rllib.core.rl_module import RLModule


class MARWILConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or MARWIL)
        self.lr = 1e-4
        self.beta = 1.0
        self.vf_coeff = 1.0
        self.moving_average_sqd_adv_norm_start = 100.0
        self.moving_average_sqd_adv_norm_update_rate = 1e-8
        self.train_batch_size = 2000
        self.num_env_runners = 0
        self.updates_per_iteration = 10
        self.eval_steps_per_iteration = 500
        self.grad_clip = None
        self.model = {"fcnet_hiddens": [256, 256], "fcnet_activation": "tanh"}


class BCConfig(MARWILConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or BC)
        self.beta = 0.0
        self.vf_coeff = 0.0


class MARWILLearner(TorchLearner):
    """MARWIL / BC on the learner pipeline (reference: marwil/torch/
    marwil_torch_learner.py). The running mean of squared advantages is a learner-side
    statistic: with several learners it is updated from the group-wide batch mean, so
    every rank keeps the same value (and the same weights)."""

    def build_module(self):
        self.ma_sqd = float(self.config.get("moving_average_sqd_adv_norm_start", 100.0))
        return RLModule(self.observation_space, self.action_space, self.config.get("model"))

    def configure_optimizers_for_module(self, module_id, config):
        params = list(self.module.parameters())
        self.register_optimizer(module_id=module_id, optimizer=torch.optim.Adam(
            params, lr=config.get("lr", 1e-4)), params=params)

    def _logp(self, di, actions):
        m = self.module
        if m.discrete:
            return torch.log_softmax(di.float(), -1).gather(-1, actions.long()[:, None])[:, 0]
        from ray_amd.rllib.core.rl_module import gaussian_logp

        mean, log_std = di.float().chunk(2, -1)
        return gaussian_logp(actions.float(), mean, log_std)

    def compute_loss_for_module(self, *, module_id, config, batch, fwd_out):
        logp = self._logp(fwd_out["action_dist_inputs"], batch["actions"])
        beta = float(config.get("beta", 1.0))
        self.metrics = {}
        if beta == 0.0:  # BC: plain negative log-likelihood
            loss = -logp.mean()
            self.metrics["policy_loss"] = float(loss.detach())
            return loss
        v = fwd_out["vf_preds"].float()
        adv = batch["returns"].float() - v
        with torch.no_grad():
            rate = float(config.get("moving_average_sqd_adv_norm_update_rate", 1e-8))
            sq = self._allreduce_mean(float((adv.detach() ** 2).mean()))
            self.ma_sqd += rate * (sq - self.ma_sqd)
            w = torch.exp(beta * adv.detach() / (1e-8 + self.ma_sqd ** 0.5)).clamp(max=20.0)
        pi_loss = -(w * logp).mean()
        vf_loss = 0.5 * (adv ** 2).mean()
        self.metrics.update(policy_loss=float(pi_loss.detach()),
                            vf_loss=float(vf_loss.detach()))
        return pi_loss + float(config.get("vf_coeff", 1.0)) * vf_loss

    def _extra_state(self):
        return {"ma": self.ma_sqd}

    def _load_extra_state(self, s):
        self.ma_sqd = s.get("ma", self.ma_sqd)


class MARWIL(Algorithm):
    @classmethod
    def get_default_config(cls):
        return MARWILConfig()

    def setup(self):
        self._setup_offline()
        self.learner_group = LearnerGroup(self.cfg, self.observation_space, self.action_space,
                                          learner_class=MARWILLearner)
        self._sync_weights(self.learner_group.get_weights())

    def training_step(self):
        cfg = self.config
        stats = self._offline_updates(int(cfg.updates_per_iteration), int(cfg.train_batch_size))
        stats = {k: v for k, v in stats.items() if not isinstance(v, np.ndarray)}
        self._sync_weights(self.learner_group.get_weights())
        if cfg.eval_steps_per_iteration:  # online metrics with the current policy
            runner = self.env_runners[0] if self.env_runners else self.local_runner
            n = max(1, cfg.eval_steps_per_iteration // max(1, cfg.num_envs_per_env_runner))
            if self.env_runners:
                import ray_amd as ray

                ray.get(runner.sample.remote(n, False))
            else:
                runner.sample(n, explore=False)
        return stats


class BC(MARWIL):
    @classmethod
    def get_default_config(cls):
        return BCConfig()
