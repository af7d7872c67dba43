"""IMPALA and APPO (reference: rllib/algorithms/impala/impala.py, rllib/algorithms/appo).

Asynchronous sampling: every EnvRunner always has one ``sample`` request in
flight; the driver feeds finished fragments to the learner as they arrive and
broadcasts fresh weights every ``broadcast_interval`` updates. The learner
corrects the policy lag with V-trace (HIP reverse-scan kernel)."""

from __future__ import annotations

import ray_amd as ray
from ray_amd.rllib.algorithms.algorithm import Algorithm
from ray_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_amd.rllib.core.learner import LearnerGroup


class IMPALAConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or IMPALA)
        self.rollout_fragment_length = 50
        self.train_batch_size = 500
        self.lr = 5e-4
        self.vtrace_clip_rho_threshold = 1.0
        self.vtrace_clip_pg_rho_threshold = 1.0
        self.vf_loss_coeff = 0.5
        self.entropy_coeff = 0.01
        self.broadcast_interval = 1
        self.grad_clip = 40.0
        self.appo = False


class IMPALA(Algorithm):
    kind = "vtrace"
    supports_multi_agent = True

    @classmethod
    def get_default_config(cls):
        return IMPALAConfig()

    def setup(self):
        if self.is_multi_agent:  # one V-trace learner per trainable module
            from ray_amd.rllib.core.learner import MultiAgentLearnerGroup

            self.learner_group = MultiAgentLearnerGroup(self.cfg, self.module_specs,
                                                        self.config.policies_to_train)
        else:
            self.learner_group = LearnerGroup(self.cfg, self.observation_space,
                                              self.action_space)
        self._sync_weights(self.learner_group.get_weights())
        self._inflight = {}
        self._updates = 0

    def training_step(self) -> dict:
        cfg = self.config
        if not self.env_runners:
            b = self.local_runner.sample(cfg.rollout_fragment_length)
            self.total_env_steps += b["env_steps"]
            stats = self.learner_group.update("vtrace", [b])
            self._sync_weights(self.learner_group.get_weights())
            return stats
        self._metrics_from_samples = True
        for r in self.env_runners:
            if r not in self._inflight.values():
                self._inflight[r.sample.remote(cfg.rollout_fragment_length,
                                               with_metrics=True)] = r
        need = max(1, cfg.train_batch_size // (cfg.rollout_fragment_length *
                                                cfg.num_envs_per_env_runner))
        batches = []
        stats = {}
        while len(batches) < need:
            ready, _ = ray.wait(list(self._inflight), num_returns=1)
            ref = ready[0]
            runner = self._inflight.pop(ref)
            b = ray.get(ref)
            self._take_metrics(b)
            self.total_env_steps += b["env_steps"]
            batches.append(b)
            self._inflight[runner.sample.remote(cfg.rollout_fragment_length,
                                                with_metrics=True)] = runner
        stats = self.learner_group.update("vtrace", batches)
        self._updates += 1
        if self._updates % cfg.broadcast_interval == 0:
            w = self.learner_group.get_weights()
            self.weights_version += 1
            ref = ray.put(w)
            for r in self.env_runners:
                r.set_weights.remote(ref, self.weights_version)
        return stats


class APPOConfig(IMPALAConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or APPO)
        self.appo = True
        self.clip_param = 0.4
        self.lr = 5e-4


class APPO(IMPALA):
    @classmethod
    def get_default_config(cls):
        return APPOConfig()
