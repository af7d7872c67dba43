"""DQN (double, dueling, prioritized replay, n-step=1) (reference: rllib/algorithms/dqn/)."""

from __future__ import annotations

import numpy as np
import torch

import ray_amd as ray
from ray_amd.rllib.algorithms.algorithm import (Algorithm, PerModuleLearners, add_agent_rows,
                                                 flat_transitions)
from ray_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_amd.rllib.core.learner import LearnerGroup, TorchLearner
from ray_amd.rllib.core.rl_module import QModule
from ray_amd.rllib.utils.replay_buffers import PrioritizedReplayBuffer, ReplayBuffer


class DQNConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or DQN)
        self.lr = 5e-4
        self.train_batch_size = 32
        self.rollout_fragment_length = 4
        self.num_env_runners = 0
        self.replay_buffer_config = {"type": "PrioritizedEpisodeReplayBuffer", "capacity": 50000,
                                     "alpha": 0.6, "beta": 0.4}
        self.num_steps_sampled_before_learning_starts = 1000
        self.target_network_update_freq = 500
        self.double_q = True
        self.dueling = True
        self.epsilon = [(0, 1.0), (10000, 0.05)]
        self.training_intensity = None
        self.grad_clip = 40.0
        self.model = {"fcnet_hiddens": [256], "fcnet_activation": "relu"}
        self.n_step = 1


class DQNLearner(TorchLearner):
    """DQN on the learner pipeline (reference: rllib/algorithms/dqn/torch/
    dqn_torch_learner.py): forward_train evaluates Q(s, a) and the (double-)Q target from
    the target network, the loss is the importance-weighted Huber TD error, the target
    network is synced by ``sync_target``; per-row |TD| comes back as ``td_error`` for the
    prioritized replay buffer. ``num_learners=N``: N learners on 1/N of each batch."""

    def build_module(self):
        mc = dict(self.config.get("model") or {})
        mc["dueling"] = self.config.get("dueling", True)
        m = torch.nn.ModuleDict({"q": QModule(self.observation_space, self.action_space, mc),
                                 "target": QModule(self.observation_space, self.action_space,
                                                   mc)})
        m["target"].load_state_dict(m["q"].state_dict())
        m["target"].requires_grad_(False)
        return m

    def configure_optimizers_for_module(self, module_id, config):
        params = list(self.module["q"].parameters())
        self.register_optimizer(module_id=module_id, optimizer=torch.optim.Adam(
            params, lr=config.get("lr", 5e-4)), params=params)

    def forward_train(self, b):
        q = self.module["q"]
        qa = q(b["obs"]).gather(-1, b["actions"].long()[:, None])[:, 0]
        with torch.no_grad():
            nobs = b["next_obs"]
            if self.config.get("double_q", True):
                na = q(nobs).argmax(-1)
                nq = self.module["target"](nobs).gather(-1, na[:, None])[:, 0]
            else:
                nq = self.module["target"](nobs).max(-1).values
            disc = b["discounts"].float() if "discounts" in b else \
                self.config.get("gamma", 0.99)  # n-step rows carry gamma ** k
            tgt = b["rewards"].float() + disc * (1 - b["terminateds"].float()) * nq
        return {"q": qa, "target": tgt}

    def compute_loss_for_module(self, *, module_id, config, batch, fwd_out):
        q, tgt = fwd_out["q"], fwd_out["target"]
        w = batch.get("weights")
        self._td = (q - tgt).detach()
        hub = torch.nn.functional.huber_loss(q, tgt, reduction="none")
        return (hub * w.float()).mean() if w is not None else hub.mean()

    def _update(self, batch, timesteps=None):
        out = super()._update(batch, timesteps=timesteps)
        out["loss"] = out["total_loss"]
        out["td_error"] = self._td.abs().float().cpu().numpy()
        return out

    def sync_target(self):
        self.module["target"].load_state_dict(self.module["q"].state_dict())

    # the EnvRunners run the online Q network: its state dict is "the weights"
    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.module["q"].state_dict().items()}

    def set_weights(self, w):
        self.module["q"].load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})
        self.sync_target()


_QLearner = DQNLearner  # earlier name


class DQN(Algorithm):
    """DQN. ``replay_buffer_config={"type": "EpisodeReplayBuffer"}`` makes the EnvRunners
    return SingleAgentEpisodes that an EpisodeReplayBuffer stores whole and samples as
    ``n_step`` transitions (reference: dqn.py new API stack); other types keep the
    transition-level (prioritized) buffer."""

    module_kind = "q"
    supports_multi_agent = True

    def __init__(self, config):
        t = (config.replay_buffer_config or {}).get("type", "")
        t = t if isinstance(t, str) else getattr(t, "__name__", "")
        self.episodic = t == "EpisodeReplayBuffer" and not config.is_multi_agent
        config._record_episodes = self.episodic
        super().__init__(config)

    @classmethod
    def get_default_config(cls):
        return DQNConfig()

    def _new_buffer(self):
        rb = self.config.replay_buffer_config
        cap = rb.get("capacity", 50000)
        if self.episodic:
            from ray_amd.rllib.utils.replay_buffers.episode_replay_buffer import \
                EpisodeReplayBuffer

            return EpisodeReplayBuffer(cap, seed=self.config.seed)
        return PrioritizedReplayBuffer(cap, rb.get("alpha", 0.6), self.config.seed) \
            if self.prioritized else ReplayBuffer(cap, self.config.seed)

    def setup(self):
        t = self.config.replay_buffer_config.get("type", "")
        self.prioritized = "Prioritized" in (t if isinstance(t, str) else "") and \
            not self.episodic
        if self.is_multi_agent:
            self.learner_group = PerModuleLearners(
                lambda os_, as_, mid: LearnerGroup(self.cfg, os_, as_, module_id=mid,
                                                   learner_class=DQNLearner),
                self.module_specs, self.config.policies_to_train)
            self.buffers = {mid: self._new_buffer() for mid in self.learner_group.trainable}
        else:
            self.buffer = self._new_buffer()
            self.learner_group = LearnerGroup(self.cfg, self.observation_space,
                                              self.action_space, learner_class=DQNLearner)
        self._last_target = 0
        self._sync_weights(self.learner_group.get_weights())

    def _add_multi_agent(self, b):
        add_agent_rows(self.buffers, b)
        self.total_env_steps += b["env_steps"]

    def _train_multi_agent(self, n_updates, stats):
        cfg = self.config
        for mid, buf in self.buffers.items():
            if len(buf) < cfg.train_batch_size:
                continue
            for _ in range(n_updates):
                kw = {"beta": cfg.replay_buffer_config.get("beta", 0.4)} \
                    if self.prioritized else {}
                mb = buf.sample(cfg.train_batch_size, **kw)
                res = self.learner_group.learners[mid].update_from_batch(
                    mb, timesteps=self.total_env_steps)
                if self.prioritized:
                    buf.update_priorities(mb["batch_indexes"], res["td_error"])
                stats[f"{mid}/loss"] = res["loss"]

    def _epsilon(self):
        sched = self.config.epsilon
        t = self.total_env_steps
        (t0, e0), (t1, e1) = sched[0], sched[-1]
        if t >= t1:
            return e1
        return e0 + (e1 - e0) * (t - t0) / max(1, t1 - t0)

    def training_step(self):
        cfg = self.config
        eps = self._epsilon()
        if self._runners.num_actors():
            bs = self._foreach_runner(lambda r: r.sample.remote(cfg.rollout_fragment_length,
                                                                True, eps))
        else:
            bs = [self.local_runner.sample(cfg.rollout_fragment_length, True, eps)]
        for b in bs:
            if self.is_multi_agent:
                self._add_multi_agent(b)
                continue
            if self.episodic:
                self.buffer.add(b["episodes"])
                self.total_env_steps += b["env_steps"]
                continue
            flat = flat_transitions(b)
            self.buffer.add(flat)
            self.total_env_steps += len(flat["rewards"])
        stats = {"epsilon": eps}
        if self.total_env_steps < cfg.num_steps_sampled_before_learning_starts:
            return stats
        sampled = sum(b["env_steps"] for b in bs)
        if cfg.training_intensity:  # replay ratio: trained rows per sampled env step
            n_updates = max(1, int(round(sampled * cfg.training_intensity /
                                         cfg.train_batch_size)))
        else:
            n_updates = max(1, sampled // max(1, cfg.rollout_fragment_length))
        if self.is_multi_agent:
            self._train_multi_agent(n_updates, stats)
            n_updates = 0
        for _ in range(n_updates):
            kw = {"beta": cfg.replay_buffer_config.get("beta", 0.4)} if self.prioritized else {}
            if self.episodic:
                kw = {"n_step": int(getattr(cfg, "n_step", 1) or 1), "gamma": cfg.gamma}
            mb = self.buffer.sample(cfg.train_batch_size, **kw)
            res = self.learner_group.update_from_batch(mb, timesteps=self.total_env_steps)
            if self.prioritized:
                self.buffer.update_priorities(mb["batch_indexes"], res["td_error"])
            stats["loss"] = res["loss"]
        if self.total_env_steps - self._last_target >= cfg.target_network_update_freq:
            self.learner_group.sync_target()
            self._last_target = self.total_env_steps
        self._sync_weights(self.learner_group.get_weights())
        return stats
