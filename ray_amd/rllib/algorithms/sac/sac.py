"""Soft Actor-Critic (reference: rllib/algorithms/sac/sac.py, sac_learner.py,
torch/sac_torch_learner.py; Haarnoja et al. 2018 with automatic entropy tuning).

Off-policy loop shared with DQN's structure: env-runner actors sample with the
squashed-Gaussian actor, transitions go to a (prioritised) replay buffer, and the
learner GPU runs critic / actor / temperature updates with Polyak-averaged target
critics. ``CQL`` (offline) subclasses the learner (``cql.py``)."""

from __future__ import annotations

import copy

import numpy as np
import torch

import ray_amd as ray
from ray_amd.rllib.algorithms.algorithm import (Algorithm, PerModuleLearners, add_agent_rows,
                                                 flat_transitions)
from ray_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_amd.rllib.core.learner import LearnerGroup, TorchLearner
from ray_amd.rllib.core.rl_module import SquashedGaussianPolicy, TwinQ
from ray_amd.rllib.utils.replay_buffers import PrioritizedReplayBuffer, ReplayBuffer


class SACConfig(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or SAC)
        self.lr = None
        self.actor_lr = 3e-4
        self.critic_lr = 3e-4
        self.alpha_lr = 3e-4
        self.train_batch_size = 256
        self.rollout_fragment_length = 1
        self.num_env_runners = 0
        self.tau = 5e-3
        self.initial_alpha = 1.0
        self.target_entropy = "auto"
        self.n_step = 1
        self.twin_q = True
        self.replay_buffer_config = {"type": "ReplayBuffer", "capacity": 100000}
        self.num_steps_sampled_before_learning_starts = 1500
        self.training_intensity = None
        self.target_network_update_freq = 0
        self.grad_clip = None
        self.bootstrap_truncated = True  # time-limit truncation is not termination
        self.model = {"fcnet_hiddens": [256, 256], "fcnet_activation": "relu"}
        self.policy_model_config = None
        self.q_model_config = None


class _SACModule(torch.nn.Module):
    """The SAC networks of one learner: squashed-Gaussian actor, twin Q critics, their
    Polyak-averaged targets and the entropy temperature log(alpha)."""

    def __init__(self, cfg, obs_space, act_space):
        super().__init__()
        pm = cfg.get("policy_model_config") or cfg.get("model")
        qm = cfg.get("q_model_config") or cfg.get("model")
        self.pi = SquashedGaussianPolicy(obs_space, act_space, pm)
        self.q = TwinQ(obs_space, act_space, qm)
        self.q_t = copy.deepcopy(self.q)
        self.q_t.requires_grad_(False)
        self.log_alpha = torch.nn.Parameter(
            torch.tensor(float(np.log(cfg.get("initial_alpha", 1.0)))))


class SACLearner(TorchLearner):
    """SAC on the learner pipeline (reference: rllib/algorithms/sac/sac_learner.py,
    torch/sac_torch_learner.py): ``compute_losses`` returns the critic, actor and
    temperature losses keyed by their optimizers' names, so ``compute_gradients``
    back-propagates each into its own parameters only (the actor's loss does not touch
    the critics' gradients); gradients of every learner of the group are averaged before
    the three optimizers step; the target critics follow by Polyak averaging in
    ``after_gradient_based_update``. CQL overrides ``extra_critic_loss`` / ``actor_loss``."""

    def build_module(self):
        return _SACModule(self.config, self.observation_space, self.action_space)

    def configure_optimizers_for_module(self, module_id, config):
        m = self.module
        fused = self.device.type == "cuda"
        act_dim = int(np.prod(self.action_space.shape))
        te = config.get("target_entropy", "auto")
        self.target_entropy = -float(act_dim) if te in (None, "auto") else float(te)
        self.gamma = config.get("gamma", 0.99)
        self.tau = config.get("tau", 5e-3)
        self.register_optimizer(module_id=module_id, optimizer_name="critic",
                                optimizer=torch.optim.Adam(m.q.parameters(),
                                                           lr=config.get("critic_lr", 3e-4),
                                                           fused=fused),
                                params=list(m.q.parameters()))
        self.register_optimizer(module_id=module_id, optimizer_name="actor",
                                optimizer=torch.optim.Adam(m.pi.parameters(),
                                                           lr=config.get("actor_lr", 3e-4),
                                                           fused=fused),
                                params=list(m.pi.parameters()))
        self.register_optimizer(module_id=module_id, optimizer_name="alpha",
                                optimizer=torch.optim.Adam([m.log_alpha],
                                                           lr=config.get("alpha_lr", 3e-4)),
                                params=[m.log_alpha])

    # convenience views (CQL, tests)
    @property
    def pi(self):
        return self.module.pi

    @property
    def q(self):
        return self.module.q

    @property
    def q_t(self):
        return self.module.q_t

    @property
    def log_alpha(self):
        return self.module.log_alpha

    def _convert_batch(self, batch):
        keep = ("obs", "next_obs", "actions", "rewards", "terminateds", "weights")
        return super()._convert_batch({k: np.asarray(v) if not torch.is_tensor(v) else v
                                       for k, v in batch.items() if k in keep})

    # ---------------------------------------------------------------- losses
    def critic_target(self, b):
        with torch.no_grad():
            na, nlogp = self.pi(b["next_obs"])
            q1, q2 = self.q_t(b["next_obs"], na)
            alpha = self.log_alpha.exp()
            v = torch.min(q1, q2) - alpha * nlogp
            return b["rewards"].float() + self.gamma * (1 - b["terminateds"].float()) * v

    def extra_critic_loss(self, b, q1, q2):
        return None  # CQL adds its conservative regulariser here

    def actor_loss(self, b, a, logp, qmin, alpha):
        return (alpha * logp - qmin).mean()

    def forward_train(self, b):
        tgt = self.critic_target(b)
        q1, q2 = self.q(b["obs"], b["actions"])
        a, logp = self.pi(b["obs"])
        qa1, qa2 = self.q(b["obs"], a)
        return {"target": tgt, "q1": q1, "q2": q2, "a": a, "logp": logp,
                "qmin_pi": torch.min(qa1, qa2)}

    def compute_losses(self, *, fwd_out, batch):
        f, b = fwd_out, batch
        w = b.get("weights")
        tgt, q1, q2 = f["target"], f["q1"], f["q2"]
        self._td = (q1 - tgt).detach()
        l1, l2 = (q1 - tgt) ** 2, (q2 - tgt) ** 2
        if w is not None:
            l1, l2 = l1 * w, l2 * w
        critic = 0.5 * (l1.mean() + l2.mean())
        extra = self.extra_critic_loss(b, q1, q2)
        if extra is not None:
            critic = critic + extra
        alpha = self.log_alpha.exp().detach()
        actor = self.actor_loss(b, f["a"], f["logp"], f["qmin_pi"], alpha)
        alpha_loss = -(self.log_alpha * (f["logp"].detach() + self.target_entropy)).mean()
        self.metrics = {"alpha_value": float(alpha), "mean_q": float(q1.detach().mean()),
                        "entropy": float(-f["logp"].detach().mean())}
        return {"critic": critic, "actor": actor, "alpha": alpha_loss}

    def after_gradient_based_update(self, *, timesteps=None):
        with torch.no_grad():  # Polyak target update
            for pt, p in zip(self.q_t.parameters(), self.q.parameters()):
                pt.lerp_(p, self.tau)

    def _update(self, batch, timesteps=None):
        out = super()._update(batch, timesteps=timesteps)
        out["td_error"] = self._td.abs().float().cpu().numpy()
        return out

    # the EnvRunners run the actor: its state dict is "the weights"
    def get_weights(self):
        return {k: v.detach().cpu() for k, v in self.pi.state_dict().items()}

    def set_weights(self, w):
        self.pi.load_state_dict({k: torch.as_tensor(v) for k, v in w.items()})


class SAC(Algorithm):
    module_kind = "sac"
    learner_class = SACLearner
    supports_multi_agent = True

    @classmethod
    def get_default_config(cls):
        return SACConfig()

    def _new_buffer(self):
        rb = self.config.replay_buffer_config
        cap = rb.get("capacity", 100000)
        return PrioritizedReplayBuffer(cap, rb.get("alpha", 0.6), self.config.seed) \
            if self.prioritized else ReplayBuffer(cap, self.config.seed)

    def setup(self):
        self.prioritized = "Prioritized" in self.config.replay_buffer_config.get("type", "")
        if self.is_multi_agent:  # one SAC learner group + replay buffer per module
            self.learner_group = PerModuleLearners(
                lambda os_, as_, mid: LearnerGroup(self.cfg, os_, as_, module_id=mid,
                                                   learner_class=self.learner_class),
                self.module_specs, self.config.policies_to_train)
            self.buffers = {mid: self._new_buffer() for mid in self.learner_group.trainable}
        else:
            self.buffer = self._new_buffer()
            self.learner_group = LearnerGroup(self.cfg, self.observation_space,
                                              self.action_space, learner_class=self.learner_class)
        self._sync_weights(self.learner_group.get_weights())

    def _updates(self, buf, learner, new, stats, prefix=""):
        cfg = self.config
        if len(buf) < cfg.train_batch_size:
            return
        # reference default: one gradient step per sampled env step (training_intensity 1)
        ti = cfg.training_intensity or cfg.train_batch_size
        n_updates = max(1, int(round(new * ti / cfg.train_batch_size)))
        for _ in range(n_updates):
            kw = {"beta": cfg.replay_buffer_config.get("beta", 0.4)} if self.prioritized else {}
            mb = buf.sample(cfg.train_batch_size, **kw)
            st = learner.update_from_batch(mb, timesteps=self.total_env_steps)
            if self.prioritized:
                buf.update_priorities(mb["batch_indexes"], st["td_error"])
        stats.update({prefix + k: v for k, v in st.items() if not isinstance(v, np.ndarray)})

    def training_step(self):
        cfg = self.config
        frag = max(1, cfg.rollout_fragment_length)
        if self._runners.num_actors():
            bs = self._foreach_runner(lambda r: r.sample.remote(frag))
        else:
            bs = [self.local_runner.sample(frag)]
        new = 0
        for b in bs:
            if self.is_multi_agent:
                add_agent_rows(self.buffers, b)
                new += b["env_steps"]
                continue
            flat = flat_transitions(b)
            self.buffer.add(flat)
            new += len(flat["rewards"])
        self.total_env_steps += new
        stats = {}
        if self.total_env_steps < cfg.num_steps_sampled_before_learning_starts:
            return stats
        if self.is_multi_agent:
            for mid, buf in self.buffers.items():
                self._updates(buf, self.learner_group.learners[mid], new, stats, f"{mid}/")
        else:
            self._updates(self.buffer, self.learner_group, new, stats)
        self._sync_weights(self.learner_group.get_weights())
        return stats

    def compute_single_action(self, obs, explore=False, policy_id=None):
        a = super().compute_single_action(obs, explore, policy_id)
        return np.asarray(a, np.float32).reshape(self.action_space.shape) \
            if not self.is_multi_agent else a

    compute_action = compute_single_action
