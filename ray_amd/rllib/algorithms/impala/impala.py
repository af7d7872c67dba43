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
        # remote learners: the update runs while the next batch is sampled (one update in
        # flight; reference: IMPALA's learner thread / LearnerGroup async_update)
        self.learner_async_update = True


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
        self._inflight = {}  # meta ref -> (runner id, batch ref)
        self._updates = 0
        self._pending_update = None
        self.num_driver_batch_fetches = 0  # frame batches ray.get'd by the driver

    def _submit(self, aid):
        r = self._runners.get(aid)
        b, m = r.sample_with_meta.options(num_returns=2).remote(
            self.config.rollout_fragment_length)
        self._inflight[m] = (aid, b)

    def _broadcast(self):
        self.weights_version += 1
        ref = ray.put(self.learner_group.get_weights())
        self._last_weights_ref = ref
        for r in self.env_runners:
            r.set_weights.remote(ref, self.weights_version)

    def training_step(self) -> dict:
        cfg = self.config
        if not self._runners.num_actors():
            b = self.local_runner.sample(cfg.rollout_fragment_length)
            self.total_env_steps += b["env_steps"]
            stats = self.learner_group.update("vtrace", [b])
            self._sync_weights(self.learner_group.get_weights())
            return stats
        self._metrics_from_samples = True
        busy = {aid for aid, _ in self._inflight.values()}
        for aid in self._runners.healthy_actor_ids():
            if aid not in busy:
                self._submit(aid)
        need = max(1, cfg.train_batch_size // (cfg.rollout_fragment_length *
                                                cfg.num_envs_per_env_runner))
        refs = []
        while len(refs) < need:
            if not self._inflight:
                raise RuntimeError("IMPALA: no EnvRunner left to sample from")
            ready, _ = ray.wait(list(self._inflight), num_returns=1)
            aid, bref = self._inflight.pop(ready[0])
            try:
                meta = ray.get(ready[0])  # env steps + metrics only: the batch stays put
            except Exception as e:  # noqa: BLE001
                from ray_amd.rllib.utils.actor_manager import CallResult, _is_actor_failure

                if not _is_actor_failure(e):
                    raise
                self._runners.set_actor_state(aid, False)
                self._on_runner_failures([CallResult(aid, False, e)])
                busy = {a for a, _ in self._inflight.values()}
                for a2 in self._runners.healthy_actor_ids():
                    if a2 not in busy:
                        self._submit(a2)
                continue
            self._take_metrics(meta)
            self.total_env_steps += meta["env_steps"]
            refs.append(bref)
            self._submit(aid)
        lg = self.learner_group
        stats = {}
        if getattr(lg, "remote", False) and len(refs) >= len(lg.actors):
            if self._pending_update is not None:  # one update in flight: wait for it
                stats = lg.collect_async(self._pending_update, block=True) or {}
                self._pending_update = None
                self._after_update()
            if cfg.learner_async_update:
                self._pending_update = lg.update_from_refs("vtrace", refs, async_update=True)
            else:
                stats = lg.update_from_refs("vtrace", refs)
                self._after_update()
        else:
            self.num_driver_batch_fetches += len(refs)
            stats = lg.update("vtrace", ray.get(refs))
            self._after_update()
        return stats

    def _after_update(self):
        self._updates += 1
        if self._updates % self.config.broadcast_interval == 0:
            self._broadcast()


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
