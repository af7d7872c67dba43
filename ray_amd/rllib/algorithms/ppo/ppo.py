"""PPO (reference: rllib/algorithms/ppo/ppo.py, ppo_torch_learner.py)."""

from __future__ import annotations

import time

import ray_amd as ray
from ray_amd.rllib.algorithms.algorithm import Algorithm
from ray_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_amd.rllib.core.learner import LearnerGroup


class PPOConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or PPO)
        self.lr = 5e-5
        self.rollout_fragment_length = "auto"
        self.train_batch_size = 4000
        self.minibatch_size = 128
        self.num_epochs = 30
        self.lambda_ = 1.0
        self.use_gae = True
        self.use_critic = True
        self.use_kl_loss = True
        self.kl_coeff = 0.2
        self.kl_target = 0.01
        self.vf_loss_coeff = 1.0
        self.entropy_coeff = 0.0
        self.clip_param = 0.3
        self.vf_clip_param = 10.0
        self.grad_clip = None


class PPO(Algorithm):
    kind = "ppo"
    supports_multi_agent = True

    def __init__(self, config):
        if config.rollout_fragment_length == "auto":
            nr = max(1, config.num_env_runners) * config.num_envs_per_env_runner
            config.rollout_fragment_length = max(1, config.train_batch_size // nr)
        super().__init__(config)

    @classmethod
    def get_default_config(cls):
        return PPOConfig()

    def setup(self):
        if self.is_multi_agent:
            from ray_amd.rllib.core.learner import MultiAgentLearnerGroup

            self.learner_group = MultiAgentLearnerGroup(self.cfg, self.module_specs,
                                                        self.config.policies_to_train)
        else:
            self.learner_group = LearnerGroup(self.cfg, self.observation_space,
                                              self.action_space)
        self._sync_weights(self.learner_group.get_weights())

    def training_step(self) -> dict:
        if self.config.sample_async and self.env_runners:
            return self._training_step_async()
        t0 = time.perf_counter()
        batches = self._sample(self.config.train_batch_size)
        t1 = time.perf_counter()
        stats = self.learner_group.update("ppo", batches)
        t2 = time.perf_counter()
        self._sync_weights(self.learner_group.get_weights())
        stats = dict(stats, sample_time_s=t1 - t0, learn_time_s=t2 - t1,
                     sync_time_s=time.perf_counter() - t2)
        return stats

    def _launch_round(self):
        per = self.config.rollout_fragment_length
        return [r.sample.remote(per, with_metrics=True) for r in self.env_runners]

    def _get_round(self, pending):
        """Results of one sampling round; a runner that died mid-round is handled per
        fault_tolerance (its fragment is dropped)."""
        out, dead = [], False
        for ref in pending:
            try:
                out.append(ray.get(ref))
            except Exception as e:  # noqa: BLE001
                from ray_amd.rllib.utils.actor_manager import _is_actor_failure

                if not _is_actor_failure(e):
                    raise
                dead = True
        if dead:
            for aid in self._runners.healthy_actor_ids():
                try:
                    ray.get(self._runners.get(aid).ping.remote(), timeout=5)
                except Exception:  # noqa: BLE001
                    self._runners.set_actor_state(aid, False)
            from ray_amd.rllib.utils.actor_manager import CallResult
            from ray_amd.exceptions import ActorDiedError

            self._on_runner_failures([CallResult(0, False, ActorDiedError("EnvRunner died"))])
        return out

    def _training_step_async(self) -> dict:
        """Overlapped sampling (``sample_async``): the runners already sample batch k+1
        while the learner updates on batch k; fresh weights are queued behind that
        sample, so each batch is collected by the policy of one iteration earlier."""
        self._metrics_from_samples = True
        total = self.config.train_batch_size
        t0 = time.perf_counter()
        pending = self.__dict__.pop("_pending_round", None) or self._launch_round()
        batches, got = [], 0
        while True:
            for b in self._get_round(pending):
                self._take_metrics(b)
                got += b["env_steps"]
                batches.append(b)
            if got >= total:
                break
            pending = self._launch_round()
        self.total_env_steps += got
        self._pending_round = self._launch_round()  # overlaps the update below
        t1 = time.perf_counter()
        stats = self.learner_group.update("ppo", batches)
        t2 = time.perf_counter()
        self.weights_version += 1
        ref = ray.put(self.learner_group.get_weights())
        self._last_weights_ref = ref
        for r in self.env_runners:  # applied right after the in-flight sample
            r.set_weights.remote(ref, self.weights_version)
        return dict(stats, sample_wait_s=t1 - t0, learn_time_s=t2 - t1,
                    sync_time_s=time.perf_counter() - t2)
