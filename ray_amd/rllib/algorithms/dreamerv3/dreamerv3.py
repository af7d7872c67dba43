"""DreamerV3: model-based RL with a recurrent state-space world model and an actor-critic
trained purely in imagination.

Behaviour follows Hafner et al. 2023 ("Mastering Diverse Domains through World Models")
as exposed by the reference (rllib/algorithms/dreamerv3/dreamerv3.py: ``DreamerV3Config``
with ``model_size``, ``training_ratio``, ``batch_size_B``, ``batch_length_T``,
``horizon_H``, ``gae_lambda``, ``entropy_scale``, ``return_normalization_decay``, the three
learning rates and gradient clips; ``training_step`` alternating env sampling into an
episode replay buffer and replayed world-model/actor/critic updates until the replay to
env-step ratio reaches ``training_ratio``).

This implementation is PyTorch on the learner device (an MI355X when
``num_gpus_per_learner`` > 0):
  * world model: symlog-input encoder (MLP for vector observations, strided conv stack for
    images), GRU deterministic state + ``classes x categoricals`` stochastic state with 1 %
    unimix and straight-through sampling, decoder (symlog MSE), reward head (two-hot
    symlog over 255 bins), continue head; loss = prediction + 0.5 dynamics KL + 0.1
    representation KL, each KL clipped below at 1 free nat;
  * actor-critic: ``horizon_H``-step imagination from every posterior state of the batch,
    lambda-returns against a two-hot critic with an EMA slow-critic regulariser, returns
    normalised by the EMA of their 5th-95th percentile range (floor 1), actor trained by
    REINFORCE with an entropy bonus (both for discrete and continuous actions);
  * acting: one local env runner filtering its envs through the posterior each step.
"""

from __future__ import annotations

import math
import time
from types import SimpleNamespace

import numpy as np
import torch

from ray_amd.rllib.algorithms.algorithm import Algorithm
from ray_amd.rllib.core.learner import LearnerGroup, TorchLearner
from ray_amd.rllib.algorithms.algorithm_config import AlgorithmConfig
from ray_amd.rllib.env.envs import make_env

# (GRU units, MLP units, MLP layers, categoricals, classes), after the paper's Table B.1
MODEL_SIZES = {
    "nano": (32, 32, 1, 4, 4),
    "micro": (64, 64, 1, 8, 8),
    "mini": (128, 128, 2, 16, 16),
    "XS": (256, 256, 1, 32, 32),
    "S": (512, 512, 2, 32, 32),
    "M": (1024, 640, 3, 32, 32),
    "L": (2048, 768, 4, 32, 32),
    "XL": (4096, 1024, 5, 32, 32),
}


class DreamerV3Config(AlgorithmConfig):
    def __init__(self, algo_class=None):
        super().__init__(algo_class or DreamerV3)
        self.model_size = "XS"
        self.training_ratio = 1024
        self.batch_size_B = 16
        self.batch_length_T = 64
        self.horizon_H = 15
        self.gae_lambda = 0.95
        self.entropy_scale = 3e-4
        self.return_normalization_decay = 0.99
        self.world_model_lr = 1e-4
        self.actor_lr = 3e-5
        self.critic_lr = 3e-5
        self.world_model_grad_clip_by_global_norm = 1000.0
        self.critic_grad_clip_by_global_norm = 100.0
        self.actor_grad_clip_by_global_norm = 100.0
        self.symlog_obs = "auto"
        self.train_critic = True
        self.train_actor = True
        self.gamma = 0.997
        self.replay_buffer_config = {"capacity": int(1e6)}
        self.num_env_runners = 0
        self.num_envs_per_env_runner = 1
        self.rollout_fragment_length = 1
        self.use_float16 = False

    def training(self, *, model_size=None, training_ratio=None, batch_size_B=None,
                 batch_length_T=None, horizon_H=None, gae_lambda=None, entropy_scale=None,
                 return_normalization_decay=None, world_model_lr=None, actor_lr=None,
                 critic_lr=None, world_model_grad_clip_by_global_norm=None,
                 critic_grad_clip_by_global_norm=None, actor_grad_clip_by_global_norm=None,
                 symlog_obs=None, train_critic=None, train_actor=None,
                 replay_buffer_config=None, use_float16=None, **kw):
        for k, v in dict(model_size=model_size, training_ratio=training_ratio,
                         batch_size_B=batch_size_B, batch_length_T=batch_length_T,
                         horizon_H=horizon_H, gae_lambda=gae_lambda, entropy_scale=entropy_scale,
                         return_normalization_decay=return_normalization_decay,
                         world_model_lr=world_model_lr, actor_lr=actor_lr, critic_lr=critic_lr,
                         world_model_grad_clip_by_global_norm=world_model_grad_clip_by_global_norm,
                         critic_grad_clip_by_global_norm=critic_grad_clip_by_global_norm,
                         actor_grad_clip_by_global_norm=actor_grad_clip_by_global_norm,
                         symlog_obs=symlog_obs, train_critic=train_critic,
                         train_actor=train_actor, use_float16=use_float16).items():
            if v is not None:
                setattr(self, k, v)
        if replay_buffer_config is not None:
            self.replay_buffer_config = dict(self.replay_buffer_config, **replay_buffer_config)
        return super().training(**kw)


# ============================================================================ networks
def _torch():
    import torch

    return torch


def symlog(x):
    torch = _torch()
    return torch.sign(x) * torch.log1p(torch.abs(x))


def symexp(x):
    torch = _torch()
    return torch.sign(x) * (torch.exp(torch.abs(x)) - 1)


class _TwoHot:
    """Two-hot encoding over equally spaced bins in symlog space."""

    def __init__(self, device, n=255, lo=-20.0, hi=20.0):
        torch = _torch()
        self.bins = torch.linspace(lo, hi, n, device=device)
        self.n, self.lo, self.hi = n, lo, hi

    def encode(self, y):  # y: symlog-space targets [...]
        torch = _torch()
        y = y.clamp(self.lo, self.hi)
        pos = (y - self.lo) / (self.hi - self.lo) * (self.n - 1)
        k = pos.floor().long().clamp(0, self.n - 2)
        w = (pos - k.float()).unsqueeze(-1)
        out = torch.zeros(*y.shape, self.n, device=y.device)
        out.scatter_(-1, k.unsqueeze(-1), 1 - w)
        out.scatter_add_(-1, (k + 1).unsqueeze(-1), w)
        return out

    def mean(self, logits):  # expected value, back in real space
        return symexp((logits.softmax(-1) * self.bins).sum(-1))

    def loss(self, logits, y_real):
        return -(self.encode(symlog(y_real)) * logits.log_softmax(-1)).sum(-1)


def _mlp(torch, din, units, layers, dout=None):
    nn = torch.nn
    mods, d = [], din
    for _ in range(layers):
        mods += [nn.Linear(d, units, bias=False), nn.LayerNorm(units), nn.SiLU()]
        d = units
    if dout is not None:
        mods.append(nn.Linear(d, dout))
    return nn.Sequential(*mods)


def _build_nets(obs_shape, act_dim, discrete, size, device):
    torch = _torch()
    nn = torch.nn
    gru_units, units, layers, cats, classes = MODEL_SIZES[size]
    zdim = cats * classes
    image = len(obs_shape) == 3

    class Encoder(nn.Module):
        def __init__(self):
            super().__init__()
            if image:
                c = obs_shape[-1]
                d = max(16, units // 8)
                self.conv = nn.Sequential(
                    nn.Conv2d(c, d, 4, 2, 1), nn.SiLU(), nn.Conv2d(d, 2 * d, 4, 2, 1), nn.SiLU(),
                    nn.Conv2d(2 * d, 4 * d, 4, 2, 1), nn.SiLU(),
                    nn.Conv2d(4 * d, 8 * d, 4, 2, 1), nn.SiLU(), nn.AdaptiveAvgPool2d(4))
                self.out = nn.Linear(8 * d * 16, units)
            else:
                self.mlp = _mlp(torch, int(np.prod(obs_shape)), units, layers)

        def forward(self, x):
            if image:
                x = x.permute(0, 3, 1, 2).float() / 255.0 - 0.5
                return self.out(self.conv(x).flatten(1))
            return self.mlp(x)

    class Decoder(nn.Module):
        def __init__(self):
            super().__init__()
            self.n = int(np.prod(obs_shape))
            self.mlp = _mlp(torch, gru_units + zdim, units, layers, self.n)

        def forward(self, s):
            return self.mlp(s)

    class WorldModel(nn.Module):
        def __init__(self):
            super().__init__()
            self.encoder = Encoder()
            self.decoder = Decoder()
            self.pre_gru = _mlp(torch, zdim + act_dim, units, 1)
            self.gru = nn.GRUCell(units, gru_units)
            self.prior = _mlp(torch, gru_units, units, 1, zdim)
            self.post = _mlp(torch, gru_units + units, units, 1, zdim)
            self.reward = _mlp(torch, gru_units + zdim, units, layers, 255)
            self.cont = _mlp(torch, gru_units + zdim, units, layers, 1)
            self.h0 = nn.Parameter(torch.zeros(gru_units))
            nn.init.zeros_(self.reward[-1].weight)  # start predicting 0 reward
            nn.init.zeros_(self.reward[-1].bias)

        def dist_sample(self, logits):
            """Straight-through one-hot sample with 1 % unimix; returns (z flat, probs)."""
            lg = logits.view(*logits.shape[:-1], cats, classes)
            probs = 0.99 * lg.softmax(-1) + 0.01 / classes
            idx = torch.multinomial(probs.reshape(-1, classes), 1).view(*probs.shape[:-1])
            onehot = torch.nn.functional.one_hot(idx, classes).float()
            z = onehot + probs - probs.detach()
            return z.flatten(-2), probs

        def img_step(self, h, z, a):
            h = self.gru(self.pre_gru(torch.cat([z, a], -1)), h)
            z2, probs = self.dist_sample(self.prior(h))
            return h, z2, probs

        def initial(self, n):
            return self.h0.tanh().expand(n, -1).contiguous(), torch.zeros(n, zdim,
                                                                         device=self.h0.device)

    world = WorldModel().to(device)
    actor = _mlp(torch, gru_units + zdim, units, layers, act_dim * (1 if discrete else 2))
    critic = _mlp(torch, gru_units + zdim, units, layers, 255)
    nn.init.zeros_(critic[-1].weight)
    nn.init.zeros_(critic[-1].bias)
    return world, actor.to(device), critic.to(device), (gru_units, zdim, cats, classes)


def _kl(p, q):
    """KL(p || q) summed over categoricals; p, q: [..., cats, classes] probabilities."""
    torch = _torch()
    return (p * (torch.log(p + 1e-8) - torch.log(q + 1e-8))).sum((-2, -1))


# ============================================================================ env runner
class DreamerV3EnvRunner:
    """Steps ``num_envs_per_env_runner`` envs with the world model's posterior filter and
    the actor; returns per-step records for the replay buffer."""

    def __init__(self, cfg: dict, worker_index: int = 0):
        self.cfg = cfg
        n = max(1, int(cfg.get("num_envs_per_env_runner", 1)))
        self.envs = [make_env(cfg["env"], cfg.get("env_config")) for _ in range(n)]
        self.obs_space = self.envs[0].observation_space
        self.act_space = self.envs[0].action_space
        self.discrete = hasattr(self.act_space, "n")
        self.nets = None
        seed = cfg.get("seed")
        self.obs = [e.reset(seed=None if seed is None else seed + i)[0]
                    for i, e in enumerate(self.envs)]
        if seed is not None and hasattr(self.act_space, "seed"):
            # the random warm-up actions come from the action space: seeded, so a seeded
            # run replays bit for bit
            self.act_space.seed(seed + 1000 * worker_index)
        self.first = [True] * n
        self.ep_ret = [0.0] * n
        self.ep_len = [0] * n
        self.done_returns, self.done_lengths = [], []
        self.state = None
        self.prev_act = None
        self.total_steps = 0
        self.rew_in = np.zeros(n, np.float32)
        self.term = np.zeros(n, np.float32)
        self.pending_end = [False] * n
        self.prev_vec = None

    def ping(self):
        return True

    def bind(self, algo):
        self.algo = algo
        self.prev_vec = np.zeros((len(self.envs), algo.act_dim), np.float32)

    def _act(self, obs_batch, first, explore=True):
        torch = _torch()
        a = self.algo
        with torch.no_grad():
            x = torch.as_tensor(np.stack(obs_batch), device=a.device)
            x = a._prep_obs(x)
            n = x.shape[0]
            if self.state is None:
                self.state = a.world.initial(n)
                self.prev_act = torch.zeros(n, a.act_dim, device=a.device)
            h, z = self.state
            f = torch.as_tensor(first, device=a.device).unsqueeze(-1).float()
            h0, z0 = a.world.initial(n)
            h = f * h0 + (1 - f) * h
            z = f * z0 + (1 - f) * z
            pa = (1 - f) * self.prev_act
            h = a.world.gru(a.world.pre_gru(torch.cat([z, pa], -1)), h)
            e = a.world.encoder(x)
            z, _ = a.world.dist_sample(a.world.post(torch.cat([h, e], -1)))
            act, act_vec = a._policy(torch.cat([h, z], -1), explore)
            self.state = (h, z)
            self.prev_act = act_vec
        return act.cpu().numpy(), act_vec

    def sample(self, num_timesteps: int, random_actions: bool = False, explore: bool = True):
        """num_timesteps records per env: dict of [n_envs, T] arrays obs, prev_action
        (vector form), reward (received on arriving at obs), is_first, is_terminal (obs is a
        terminal state). An episode's final observation is recorded as its own step; the
        env is reset on the following step."""
        torch = _torch()
        n = len(self.envs)
        rec = {k: [] for k in ("obs", "prev_action", "reward", "is_first", "is_terminal")}
        for _ in range(num_timesteps):
            first = np.array(self.first, np.float32)
            rec["obs"].append(np.stack(self.obs))
            rec["is_first"].append(first)
            rec["prev_action"].append(self.prev_vec * (1 - first[:, None]))
            rec["reward"].append(self.rew_in * (1 - first))
            rec["is_terminal"].append(self.term.copy())
            if random_actions:
                acts = [self.act_space.sample() for _ in range(n)]
                vec = self.algo._action_vec(np.array(acts))
                self.state = None
            else:
                acts, vec_t = self._act(self.obs, list(self.first), explore)
                vec = vec_t.cpu().numpy()
            for i, e in enumerate(self.envs):
                if self.pending_end[i]:  # obs[i] was an episode's last observation
                    self.obs[i], _ = e.reset()
                    self.first[i] = True
                    self.rew_in[i], self.term[i], self.pending_end[i] = 0.0, 0.0, False
                    continue
                a_i = int(acts[i]) if self.discrete else acts[i]
                ob, r, te, tr, _ = e.step(a_i)
                self.obs[i], self.first[i] = ob, False
                self.rew_in[i], self.term[i] = float(r), float(te)
                self.ep_ret[i] += float(r)
                self.ep_len[i] += 1
                if te or tr:
                    self.pending_end[i] = True
                    self.done_returns.append(self.ep_ret[i])
                    self.done_lengths.append(self.ep_len[i])
                    self.ep_ret[i], self.ep_len[i] = 0.0, 0
            self.prev_vec = np.asarray(vec, np.float32)
            self.total_steps += n
        if self.state is not None:
            self.prev_act = torch.as_tensor(self.prev_vec, device=self.algo.device)
        return {k: np.stack(v, 1).astype(np.float32) if k != "obs" else np.stack(v, 1)
                for k, v in rec.items()}

    def get_metrics(self):
        r, ln = self.done_returns, self.done_lengths
        self.done_returns, self.done_lengths = [], []
        return {"episode_returns": r, "episode_lengths": ln, "num_env_steps": self.total_steps,
                "custom_metrics": {}}

    def stop(self):
        for e in self.envs:
            e.close()


# ============================================================================ replay
class _StreamReplay:
    """Per-env contiguous step streams (episodes concatenated; is_first marks starts);
    samples B windows of T consecutive steps (reference: EpisodeReplayBuffer)."""

    def __init__(self, capacity: int, seed=None):
        self.capacity = capacity
        self.streams: list = []
        self.rng = np.random.default_rng(seed)

    def add(self, rec: dict):
        n = rec["obs"].shape[0]
        while len(self.streams) < n:
            self.streams.append({})
        per = max(1, self.capacity // max(1, n))
        for i in range(n):
            s = self.streams[i]
            for k, v in rec.items():
                s[k] = v[i] if k not in s else np.concatenate([s[k], v[i]], 0)[-per:]

    def num_timesteps(self):
        return sum(len(s.get("reward", ())) for s in self.streams)

    def sample(self, B: int, T: int) -> dict:
        ok = [i for i, s in enumerate(self.streams) if len(s.get("reward", ())) >= T]
        out = {k: [] for k in self.streams[ok[0]]}
        for _ in range(B):
            s = self.streams[ok[self.rng.integers(len(ok))]]
            L = len(s["reward"])
            st = int(self.rng.integers(0, L - T + 1))
            for k in out:
                out[k].append(s[k][st:st + T])
        b = {k: np.stack(v) for k, v in out.items()}
        b["is_first"][:, 0] = 1.0  # every window starts a fresh filter
        return b


# ============================================================================ learner
class _Cfg(SimpleNamespace):
    """Attribute view of the algorithm's config dict (the learner runs in learner actors,
    where only the dict travels)."""


class DreamerV3Learner(TorchLearner):
    """DreamerV3 on the learner pipeline (reference: rllib/algorithms/dreamerv3/
    dreamerv3_learner.py, torch/dreamerv3_torch_learner.py): world model (RSSM encoder /
    GRU / posterior / prior / decoder / reward / continue heads), actor and critic with
    their own optimizers. One update: the world-model loss through compute_gradients ->
    postprocess_gradients (clip by ``world_model_grad_clip_by_global_norm``) ->
    apply_gradients; then dreamed trajectories from the posterior states give the critic
    and actor losses, each back-propagated into its own network (per-optimizer losses)
    and clipped by its own norm; the slow critic follows by EMA. With ``num_learners=N``
    every learner trains on B/N of each [B, T] batch, gradients averaged, and the return
    scale statistic is averaged over the group."""

    def build_module(self):
        c = self.c = _Cfg(**self.config)
        if c.seed is not None:
            torch.manual_seed(c.seed)
        obs_shape = tuple(self.observation_space.shape)
        self.discrete = hasattr(self.action_space, "n")
        self.act_dim = int(self.action_space.n) if self.discrete else \
            int(np.prod(self.action_space.shape))
        world, actor, critic, dims = _build_nets(obs_shape, self.act_dim, self.discrete,
                                                 c.model_size, self.device)
        self.gru_units, self.zdim, self.cats, self.classes = dims
        import copy

        m = torch.nn.Module()
        m.world, m.actor, m.critic = world, actor, critic
        m.slow_critic = copy.deepcopy(critic).requires_grad_(False)
        self.twohot = _TwoHot(self.device)
        self.image = len(obs_shape) == 3
        self.symlog_obs = (not self.image) if c.symlog_obs == "auto" else bool(c.symlog_obs)
        self.ret_scale = None  # EMA of the 5-95 percentile range of lambda-returns
        return m

    def configure_optimizers_for_module(self, module_id, config):
        c = self.c
        m = self.module
        for name, net, lr, eps in (("world_model", m.world, c.world_model_lr, 1e-8),
                                   ("actor", m.actor, c.actor_lr, 1e-5),
                                   ("critic", m.critic, c.critic_lr, 1e-5)):
            self.register_optimizer(module_id=module_id, optimizer_name=name,
                                    optimizer=torch.optim.Adam(net.parameters(), lr=lr, eps=eps),
                                    params=list(net.parameters()))

    @property
    def actor(self):
        return self.module.actor

    @property
    def critic(self):
        return self.module.critic

    @property
    def slow_critic(self):
        return self.module.slow_critic

    def postprocess_gradients(self, gradients_dict):
        """Clip each network's gradients by its own global norm."""
        c = self.c
        clip = {"world_model": c.world_model_grad_clip_by_global_norm,
                "actor": c.actor_grad_clip_by_global_norm,
                "critic": c.critic_grad_clip_by_global_norm}
        names = self._named_params()
        inv = {id(p): n for n, p in names.items()}
        for (_, oname), (_, ps) in self._optimizers.items():
            gs = [gradients_dict[inv[id(p)]] for p in ps if inv.get(id(p)) in gradients_dict]
            if gs and clip.get(oname):
                torch.nn.utils.clip_grad_norm_(gs, clip[oname])
        return gradients_dict

    def _update(self, b, timesteps=None):
        loss, post, stats = self._observe(b)
        self.apply_gradients(self.postprocess_gradients(
            self.compute_gradients({"world_model": loss})))
        stats["WORLD_MODEL_L_total"] = loss.item()
        losses, st2 = self._actor_critic_losses(post)
        if losses:
            self.apply_gradients(self.postprocess_gradients(self.compute_gradients(losses)))
        for k in ("critic", "actor"):
            if k in losses:
                stats[{"critic": "CRITIC_L_total", "actor": "ACTOR_L_total"}[k]] = \
                    losses[k].item()
        stats.update(st2)
        self.updates += 1
        self.after_gradient_based_update(timesteps=timesteps)
        return stats

    def after_gradient_based_update(self, *, timesteps=None):
        if self.c.train_critic:
            with torch.no_grad():  # slow critic EMA
                for ps, p in zip(self.slow_critic.parameters(), self.critic.parameters()):
                    ps.mul_(0.98).add_(p.detach(), alpha=0.02)

    def _convert_batch(self, batch):
        return batch  # _observe moves the [B, T] fields itself

    def _extra_state(self):
        return {"ret_scale": self.ret_scale}

    def _load_extra_state(self, s):
        self.ret_scale = s.get("ret_scale", self.ret_scale)

    # --- world model ----------------------------------------------------------------
    def _prep_obs(self, x):
        if self.image:
            return x
        x = x.float().flatten(1)
        return symlog(x) if self.symlog_obs else x

    def _policy(self, s, explore):
        torch = _torch()
        out = self.actor(s)
        if self.discrete:
            probs = 0.99 * out.softmax(-1) + 0.01 / self.act_dim
            idx = torch.multinomial(probs, 1).squeeze(-1) if explore else probs.argmax(-1)
            return idx, torch.nn.functional.one_hot(idx, self.act_dim).float()
        mu, log_std = out.chunk(2, -1)
        std = torch.nn.functional.softplus(log_std) + 0.1
        a = torch.tanh(mu + std * torch.randn_like(mu)) if explore else torch.tanh(mu)
        lo = torch.as_tensor(self.action_space.low, device=a.device, dtype=a.dtype)
        hi = torch.as_tensor(self.action_space.high, device=a.device, dtype=a.dtype)
        return lo + (a + 1) * 0.5 * (hi - lo), a

    def _actor_dist(self, s):
        torch = _torch()
        out = self.actor(s)
        if self.discrete:
            probs = 0.99 * out.softmax(-1) + 0.01 / self.act_dim
            return torch.distributions.OneHotCategorical(probs=probs)
        mu, log_std = out.chunk(2, -1)
        std = torch.nn.functional.softplus(log_std) + 0.1
        return torch.distributions.Independent(torch.distributions.Normal(mu, std), 1)

    # --- world model ----------------------------------------------------------------
    def _observe(self, b):
        """Posterior filter over a [B, T] batch; returns states and the losses."""
        torch = _torch()
        dev = self.device
        obs = torch.as_tensor(b["obs"], device=dev)
        B, T = obs.shape[:2]
        x = self._prep_obs(obs.reshape(B * T, *obs.shape[2:]))
        emb = self.module.world.encoder(x).view(B, T, -1)
        pa = torch.as_tensor(b["prev_action"], device=dev)
        first = torch.as_tensor(b["is_first"], device=dev).unsqueeze(-1)
        h, z = self.module.world.initial(B)
        hs, zs, post_p, prior_p = [], [], [], []
        h0, z0 = self.module.world.initial(B)
        for t in range(T):
            f = first[:, t]
            h = f * h0 + (1 - f) * h
            z = f * z0 + (1 - f) * z
            a = (1 - f) * pa[:, t]
            h = self.module.world.gru(self.module.world.pre_gru(torch.cat([z, a], -1)), h)
            prior_logits = self.module.world.prior(h)
            post_logits = self.module.world.post(torch.cat([h, emb[:, t]], -1))
            z, pp = self.module.world.dist_sample(post_logits)
            lp = prior_logits.view(B, self.cats, self.classes)
            prior_p.append(0.99 * lp.softmax(-1) + 0.01 / self.classes)
            post_p.append(pp)
            hs.append(h)
            zs.append(z)
        H_ = torch.stack(hs, 1)
        Z_ = torch.stack(zs, 1)
        post_p = torch.stack(post_p, 1)
        prior_p = torch.stack(prior_p, 1)
        s = torch.cat([H_, Z_], -1)
        recon = self.module.world.decoder(s.reshape(B * T, -1))
        target = x.float().flatten(1)
        if self.image:
            target = target / 255.0 - 0.5
        l_dec = ((recon - target) ** 2).sum(-1).view(B, T)
        rew = torch.as_tensor(b["reward"], device=dev)
        l_rew = self.twohot.loss(self.module.world.reward(s), rew)
        cont = 1.0 - torch.as_tensor(b["is_terminal"], device=dev)
        l_cont = torch.nn.functional.binary_cross_entropy_with_logits(
            self.module.world.cont(s).squeeze(-1), cont, reduction="none")
        kl_dyn = _kl(post_p.detach(), prior_p).clamp_min(1.0)
        kl_rep = _kl(post_p, prior_p.detach()).clamp_min(1.0)
        loss = (l_dec + l_rew + l_cont + 0.5 * kl_dyn + 0.1 * kl_rep).mean()
        stats = {"WORLD_MODEL_L_decoder": l_dec.mean().item(),
                 "WORLD_MODEL_L_reward": l_rew.mean().item(),
                 "WORLD_MODEL_L_continue": l_cont.mean().item(),
                 "WORLD_MODEL_L_dynamics": kl_dyn.mean().item(),
                 "WORLD_MODEL_L_representation": kl_rep.mean().item()}
        return loss, s.detach(), stats

    # --- imagination ----------------------------------------------------------------
    def _imagine(self, start):
        torch = _torch()
        H = self.c.horizon_H
        h, z = start[:, :self.gru_units], start[:, self.gru_units:]
        states, acts = [start], []
        for _ in range(H):
            s = torch.cat([h, z], -1)
            dist = self._actor_dist(s.detach())
            a = dist.sample()
            if not self.discrete:
                a = torch.tanh(a)
            acts.append(a)
            h, z, _ = self.module.world.img_step(h, z, a)
            states.append(torch.cat([h, z], -1))
        return torch.stack(states, 0), torch.stack(acts, 0)  # [H+1, N, S], [H, N, A]

    def _actor_critic_losses(self, post_states):
        """Dreamed trajectories from the posterior states -> critic / actor losses."""
        torch = _torch()
        cfg = self.c
        with torch.no_grad():
            states, acts = self._imagine(post_states.reshape(-1, post_states.shape[-1]))
            rew = self.twohot.mean(self.module.world.reward(states))  # [H+1, N]
            cont = torch.sigmoid(self.module.world.cont(states).squeeze(-1))
            disc = cfg.gamma * cont
            v_slow = self.twohot.mean(self.slow_critic(states))
        # lambda-returns from the critic (bootstrap at the horizon)
        v = self.twohot.mean(self.critic(states))
        with torch.no_grad():
            vv = v.detach()
            ret = [vv[-1]]
            for t in reversed(range(cfg.horizon_H)):
                ret.append(rew[t + 1] + disc[t + 1] * ((1 - cfg.gae_lambda) * vv[t + 1] +
                                                       cfg.gae_lambda * ret[-1]))
            ret = torch.stack(ret[::-1][:-1], 0)  # [H, N]
            w = torch.cumprod(torch.cat([torch.ones_like(disc[:1]), disc[1:-1]], 0), 0)
            lo, hi = torch.quantile(ret.flatten().float(), torch.tensor([0.05, 0.95],
                                                                        device=ret.device))
            rng = self._allreduce_mean((hi - lo).item())  # the same scale on every learner
            d = cfg.return_normalization_decay
            self.ret_scale = rng if self.ret_scale is None else d * self.ret_scale + \
                (1 - d) * rng
            scale = max(1.0, self.ret_scale)
        stats, losses = {}, {}
        if cfg.train_critic:
            logits = self.critic(states[:-1].detach())
            l_c = self.twohot.loss(logits, ret) + self.twohot.loss(logits, v_slow[:-1])
            losses["critic"] = (l_c * w).mean()
        if cfg.train_actor:
            dist = self._actor_dist(states[:-1].detach())
            a = acts if self.discrete else torch.atanh(acts.clamp(-0.999, 0.999))
            logp = dist.log_prob(a)
            adv = ((ret - vv[:-1]) / scale).detach()
            ent = dist.entropy()
            l_a = (-(logp * adv) - cfg.entropy_scale * ent) * w
            losses["actor"] = l_a.mean()
            stats["ACTOR_entropy"] = ent.mean().item()
        stats["DREAM_return_scale"] = scale
        stats["DREAM_rewards_mean"] = rew.mean().item()
        return losses, stats



# ============================================================================ algorithm
class DreamerV3(Algorithm):
    kind = "dreamerv3"
    env_runner_cls = DreamerV3EnvRunner

    @classmethod
    def get_default_config(cls):
        return DreamerV3Config()

    def setup(self):
        cfg = self.config
        if cfg.seed is not None:
            torch.manual_seed(cfg.seed)
        self.cfg["num_gpus_per_learner"] = 1 if (cfg.num_gpus_per_learner and
                                                 torch.cuda.is_available()) else 0
        self.learner_group = LearnerGroup(self.cfg, self.observation_space, self.action_space,
                                          learner_class=DreamerV3Learner)
        # the networks the EnvRunner acts with: the learner's own when it is local, else an
        # inference copy refreshed from the learners after every training step
        self._infer = self.learner_group.local if self.learner_group.is_local else \
            DreamerV3Learner(self.cfg, self.observation_space, self.action_space)
        self.device = self._infer.device
        self.discrete, self.act_dim = self._infer.discrete, self._infer.act_dim
        self.gru_units, self.zdim = self._infer.gru_units, self._infer.zdim
        self.cats, self.classes = self._infer.cats, self._infer.classes
        self.image = self._infer.image
        self.replay = _StreamReplay(int(cfg.replay_buffer_config.get("capacity", 1e6)),
                                    cfg.seed)
        self.local_runner.bind(self)
        self.replayed_steps = 0
        self.env_steps = 0
        self._sync_infer()

    # networks / helpers of the acting copy
    @property
    def world(self):
        return self._infer.module.world

    @property
    def actor(self):
        return self._infer.actor

    @property
    def critic(self):
        return self._infer.critic

    @property
    def slow_critic(self):
        return self._infer.slow_critic

    @property
    def ret_scale(self):
        return self.learner_group.foreach_learner(lambda lr: lr.ret_scale)[0]

    def _prep_obs(self, x):
        return self._infer._prep_obs(x)

    def _action_vec(self, acts):
        if self.discrete:
            return np.eye(self.act_dim, dtype=np.float32)[acts.astype(np.int64)]
        return np.asarray(acts, np.float32).reshape(len(acts), -1)

    def _policy(self, s, explore):
        return self._infer._policy(s, explore)

    def _sync_infer(self):
        if not self.learner_group.is_local:
            self._infer.module.load_state_dict(
                {k: torch.as_tensor(v) for k, v in self.learner_group.foreach_learner(
                    lambda lr: {k: v.detach().cpu() for k, v in
                                lr.module.state_dict().items()})[0].items()})

    def _update(self, b, sync=True):
        """One learner-group update on a [B, T] replay batch (then the acting copy follows
        unless ``sync=False``: the training loop syncs once per iteration)."""
        res = self.learner_group.update_from_batch(b)
        if sync:
            self._sync_infer()
        return res

    # --- training loop --------------------------------------------------------------
    def training_step(self) -> dict:
        """Sample env steps into the replay buffer (random actions until one B x T batch
        is stored), then replay B x T batches until replayed / sampled steps reaches
        ``training_ratio``."""
        cfg = self.config
        B, T = cfg.batch_size_B, cfg.batch_length_T
        t0 = time.perf_counter()
        runner = self.local_runner
        frag = max(1, int(cfg.rollout_fragment_length))
        sampled = 0
        while True:
            fill = self.replay.num_timesteps() < B * T
            rec = runner.sample(frag, random_actions=fill and self.env_steps == 0)
            self.replay.add(rec)
            sampled += rec["reward"].size
            if self.replay.num_timesteps() >= B * T:
                break
        self.env_steps += sampled
        self.total_env_steps += sampled
        t1 = time.perf_counter()
        stats, n_up = {}, 0
        while self.replayed_steps < cfg.training_ratio * self.env_steps:
            stats = self._update(self.replay.sample(B, T), sync=False)
            self.replayed_steps += B * T
            n_up += 1
        self._sync_infer()
        stats.update({"sample_time_s": t1 - t0, "learn_time_s": time.perf_counter() - t1,
                      "num_updates": n_up, "replay_timesteps": self.replay.num_timesteps(),
                      "replayed_steps": self.replayed_steps})
        return stats

    # --- inference / checkpoints ----------------------------------------------------
    def compute_single_action(self, obs, explore=False, state=None, policy_id=None):
        """One action from a fresh filter state (or ``state`` = (h, z) returned before);
        returns the action (and the new state when ``state`` is given)."""
        torch = _torch()
        with torch.no_grad():
            x = self._prep_obs(torch.as_tensor(np.asarray(obs)[None], device=self.device))
            h, z = state if state is not None else self.world.initial(1)
            h = self.world.gru(self.world.pre_gru(
                torch.cat([z, torch.zeros(1, self.act_dim, device=self.device)], -1)), h)
            z, _ = self.world.dist_sample(self.world.post(torch.cat([h, self.world.encoder(x)],
                                                                    -1)))
            a, _ = self._policy(torch.cat([h, z], -1), explore)
        out = a[0].cpu().numpy()
        out = int(out) if self.discrete else out
        return (out, (h, z)) if state is not None else out

    compute_action = compute_single_action

    def get_weights(self):
        return {"world": self.world.state_dict(), "actor": self.actor.state_dict(),
                "critic": self.critic.state_dict()}

    def get_state(self):
        return {"learner": self.learner_group.get_state(),
                "iteration": self.iteration, "total_env_steps": self.total_env_steps,
                "env_steps": self.env_steps, "replayed_steps": self.replayed_steps,
                "config": self.cfg}

    def set_state(self, s):
        self.learner_group.set_state(s["learner"])
        self._sync_infer()
        self.iteration = s["iteration"]
        self.total_env_steps = s["total_env_steps"]
        self.env_steps = s["env_steps"]
        self.replayed_steps = s["replayed_steps"]

    def stop(self):
        self.local_runner.stop()
        self.learner_group.shutdown()


DreamerV3Config.algo_class = DreamerV3
math  # noqa: B018
