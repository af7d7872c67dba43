"""RLModule + model catalog (reference: rllib/core/rl_module/rl_module.py,
rllib/core/models/catalog.py, rllib/algorithms/ppo/ppo_catalog.py,
rllib/models/torch/torch_action_dist.py).

Encoders: MLP for vector observations, Nature-CNN (Mnih et al. 2015) for image
observations ([H, W, C] uint8 frames; the /255 scaling is fused into the uint8
→ bf16 HIP cast kernel on GPU). Heads: policy logits (Categorical) or
mean/log-std (DiagGaussian) and a value head.
"""

from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn

from ray_amd.rllib.core.rl_module.checkpoint import CheckpointableModuleMixin
import torch.nn.functional as F

from ray_amd.rllib.env import spaces


def _act(name):
    return {"relu": nn.ReLU, "tanh": nn.Tanh, "swish": nn.SiLU, "silu": nn.SiLU,
            "elu": nn.ELU}.get(name or "tanh", nn.Tanh)


class MLP(nn.Module):
    def __init__(self, in_dim, hiddens, activation="tanh"):
        super().__init__()
        layers = []
        d = in_dim
        for h in hiddens:
            layers += [nn.Linear(d, h), _act(activation)()]
            d = h
        self.net = nn.Sequential(*layers)
        self.out_dim = d

    def forward(self, x):
        return self.net(x)


class NatureCNN(nn.Module):
    """Conv(32,8,4) → Conv(64,4,2) → Conv(64,3,1) → FC(512), RLlib's default Atari stack."""

    def __init__(self, obs_shape, out_dim=512):
        super().__init__()
        H, W, C = obs_shape
        self.convs = nn.Sequential(
            nn.Conv2d(C, 32, 8, 4), nn.ReLU(), nn.Conv2d(32, 64, 4, 2), nn.ReLU(),
            nn.Conv2d(64, 64, 3, 1), nn.ReLU())
        with torch.no_grad():
            n = self.convs(torch.zeros(1, C, H, W)).numel()
        self.fc = nn.Sequential(nn.Linear(n, out_dim), nn.ReLU())
        self.out_dim = out_dim

    def forward(self, x, idx=None):
        """x: [B, H, W, C] uint8 or float frames; idx: optional rows of x to encode (the
        learner's minibatch — the first conv gathers them itself on GPU)."""
        mods = list(self.convs)
        convs, acts = mods[0::2], mods[1::2]
        if x.is_cuda and convs[0].weight.dtype == torch.bfloat16:
            # GPU: MFMA NHWC implicit-GEMM convs with fused bias + ReLU (ray_amd.ops conv.hip);
            # the first layer reads the uint8 frames (and the minibatch rows) directly.
            # NHWC frames are a channels-last NCHW view, and the flatten below is NHWC
            # order: a free view of the channels-last output
            from ray_amd.ops.functional import conv2d_bias_relu

            if x.dtype != torch.uint8:
                if idx is not None:
                    x = x.index_select(0, idx)
                    idx = None
                x = x.to(torch.bfloat16).permute(0, 3, 1, 2)
            from ray_amd.ops.functional import linear_relu

            for i, conv in enumerate(convs):
                x = conv2d_bias_relu(x, conv.weight, conv.bias, conv.stride[0],
                                     idx=idx if i == 0 else None)
            fc = self.fc[0]
            return linear_relu(x.permute(0, 2, 3, 1).flatten(1), fc.weight, fc.bias)
        if idx is not None:
            x = x.index_select(0, idx)
        wdt = self.fc[0].weight.dtype
        if x.dtype == torch.uint8:
            if x.is_cuda:
                from ray_amd.ops.functional import cast_scale_u8

                x = cast_scale_u8(x).to(wdt)
            else:  # CPU env runners: bf16 weights take bf16 frames (0..255 exact in bf16)
                x = x.to(wdt if wdt == torch.bfloat16 else torch.float32).mul_(1.0 / 255.0)
        elif x.dtype != wdt:
            x = x.to(wdt)
        x = x.permute(0, 3, 1, 2)
        for conv, act in zip(convs, acts):
            x = act(conv(x))
        return self.fc(x.permute(0, 2, 3, 1).flatten(1))


class RLModule(CheckpointableModuleMixin, nn.Module):
    """Actor-critic module used by PPO / IMPALA / APPO."""

    framework = "torch"

    def __init__(self, observation_space, action_space, model_config: dict | None = None):
        super().__init__()
        cfg = dict(model_config or {})
        self.observation_space = observation_space
        self.action_space = action_space
        self.model_config = cfg
        obs_shape = tuple(observation_space.shape)
        self.is_image = len(obs_shape) == 3
        hiddens = cfg.get("fcnet_hiddens", [256, 256])
        act = cfg.get("fcnet_activation", "tanh")
        self.discrete = isinstance(action_space, spaces.Discrete)
        if self.discrete:
            self.n_out = action_space.n
        else:
            self.act_dim = int(np.prod(action_space.shape))
            self.n_out = 2 * self.act_dim
        self.vf_share = cfg.get("vf_share_layers", self.is_image)
        if self.is_image:
            self.encoder = NatureCNN(obs_shape)
            self.vf_encoder = None if self.vf_share else NatureCNN(obs_shape)
        else:
            d = int(np.prod(obs_shape))
            self.encoder = MLP(d, hiddens, act)
            self.vf_encoder = None if self.vf_share else MLP(d, hiddens, act)
        self.pi = nn.Linear(self.encoder.out_dim, self.n_out)
        self.vf = nn.Linear(self.encoder.out_dim, 1)
        nn.init.orthogonal_(self.pi.weight, 0.01)
        nn.init.zeros_(self.pi.bias)
        nn.init.orthogonal_(self.vf.weight, 1.0)
        nn.init.zeros_(self.vf.bias)

    def _flat(self, obs):
        if isinstance(obs, dict):  # the reference's batch-dict calling convention
            obs = obs["obs"]
        if self.is_image:
            return obs
        return obs.reshape(obs.shape[0], -1).float()

    def _encode(self, enc, x, idx):
        if idx is None:
            return enc(x)
        if self.is_image:  # the conv encoder gathers the rows itself
            return enc(x, idx)
        return enc(x.index_select(0, idx))

    def forward_train(self, obs, idx=None):
        """idx: optional rows of ``obs`` (a minibatch of a resident train batch)."""
        x = self._flat(obs)
        h = self._encode(self.encoder, x, idx)
        logits = self.pi(h)
        hv = h if self.vf_encoder is None else self._encode(self.vf_encoder, x, idx)
        v = self.vf(hv).squeeze(-1)
        return {"action_dist_inputs": logits, "vf_preds": v}

    def forward_inference(self, obs):
        return {"action_dist_inputs": self.pi(self.encoder(self._flat(obs)))}

    def forward_exploration(self, obs):
        return self.forward_train(obs)

    def value(self, obs):
        x = self._flat(obs)
        hv = self.encoder(x) if self.vf_encoder is None else self.vf_encoder(x)
        return self.vf(hv).squeeze(-1)

    # ---------------------------------------------------------------- distributions
    def sample_actions(self, dist_inputs, explore=True):
        """Returns (actions, logp)."""
        if self.discrete:
            lp_all = torch.log_softmax(dist_inputs.float(), -1)
            if explore:
                # Gumbel-max draw: argmax(logp + G), G = -log(-log U) ~ Gumbel(0, 1) —
                # exact categorical sampling in three ops (no Distribution object per step)
                u = torch.rand_like(lp_all).clamp_(1e-20, 1.0)
                a = (lp_all - torch.log(-torch.log(u))).argmax(-1)
            else:
                a = lp_all.argmax(-1)
            logp = lp_all.gather(-1, a[:, None])[:, 0]
            return a, logp
        mean, log_std = dist_inputs.float().chunk(2, -1)
        std = log_std.clamp(-20, 2).exp()
        a = mean + std * torch.randn_like(mean) if explore else mean
        logp = gaussian_logp(a, mean, log_std)
        return a, logp

    def get_state(self):
        return {k: v.detach().cpu() for k, v in self.state_dict().items()}

    def set_state(self, state):
        self.load_state_dict(state)

    def get_initial_state(self):
        return {}

    def is_stateful(self):
        return False


def gaussian_logp(a, mean, log_std):
    log_std = log_std.clamp(-20, 2)
    return (-0.5 * ((a - mean) / log_std.exp()) ** 2 - log_std -
            0.5 * math.log(2 * math.pi)).sum(-1)


def gaussian_entropy(log_std):
    return (log_std.clamp(-20, 2) + 0.5 * math.log(2 * math.pi * math.e)).sum(-1)


class QModule(nn.Module):
    """Q-network (optionally dueling) for DQN (reference: rllib/algorithms/dqn)."""

    def __init__(self, observation_space, action_space, model_config=None):
        super().__init__()
        cfg = dict(model_config or {})
        obs_shape = tuple(observation_space.shape)
        self.is_image = len(obs_shape) == 3
        self.dueling = cfg.get("dueling", True)
        if self.is_image:
            self.encoder = NatureCNN(obs_shape)
        else:
            self.encoder = MLP(int(np.prod(obs_shape)), cfg.get("fcnet_hiddens", [256, 256]),
                               cfg.get("fcnet_activation", "relu"))
        n = action_space.n
        self.adv = nn.Linear(self.encoder.out_dim, n)
        self.val = nn.Linear(self.encoder.out_dim, 1) if self.dueling else None

    def forward(self, obs):
        x = obs if self.is_image else obs.reshape(obs.shape[0], -1).float()
        h = self.encoder(x)
        a = self.adv(h)
        if self.val is None:
            return a
        return self.val(h) + a - a.mean(-1, keepdim=True)


class SquashedGaussianPolicy(nn.Module):
    """SAC actor: tanh-squashed diagonal Gaussian rescaled to the Box bounds
    (reference: rllib/algorithms/sac/torch/default_sac_torch_rl_module.py and
    rllib/models/torch/torch_distributions.py:TorchSquashedGaussian)."""

    def __init__(self, observation_space, action_space, model_config=None):
        super().__init__()
        cfg = dict(model_config or {})
        d = int(np.prod(observation_space.shape))
        self.act_dim = int(np.prod(action_space.shape))
        self.encoder = MLP(d, cfg.get("fcnet_hiddens", [256, 256]),
                           cfg.get("fcnet_activation", "relu"))
        self.head = nn.Linear(self.encoder.out_dim, 2 * self.act_dim)
        low = torch.tensor(np.array(action_space.low, np.float32)).reshape(-1)
        high = torch.tensor(np.array(action_space.high, np.float32)).reshape(-1)
        self.register_buffer("a_scale", (high - low) / 2)
        self.register_buffer("a_bias", (high + low) / 2)

    def forward(self, obs, explore=True, with_logp=True):
        """Returns (env-scaled actions, log pi(a|s)). Reparameterised: gradients flow."""
        h = self.encoder(obs.reshape(obs.shape[0], -1).float())
        mean, log_std = self.head(h).chunk(2, -1)
        log_std = log_std.clamp(-20, 2)
        u = mean + log_std.exp() * torch.randn_like(mean) if explore else mean
        a = torch.tanh(u)
        logp = None
        if with_logp:
            # change of variables for tanh + affine rescale (numerically stable form)
            logp = gaussian_logp(u, mean, log_std) - (
                2 * (math.log(2) - u - F.softplus(-2 * u))).sum(-1) - \
                torch.log(self.a_scale).sum()
        return a * self.a_scale + self.a_bias, logp

    def logp_of(self, obs, actions):
        """log pi(a|s) of given env-scaled actions (behaviour cloning in CQL/BC)."""
        h = self.encoder(obs.reshape(obs.shape[0], -1).float())
        mean, log_std = self.head(h).chunk(2, -1)
        log_std = log_std.clamp(-20, 2)
        a = ((actions.float() - self.a_bias) / self.a_scale).clamp(-0.999999, 0.999999)
        u = torch.atanh(a)
        return gaussian_logp(u, mean, log_std) - (
            2 * (math.log(2) - u - F.softplus(-2 * u))).sum(-1) - torch.log(self.a_scale).sum()


class TwinQ(nn.Module):
    """Q(s, a) critic pair for SAC / CQL (clipped double-Q)."""

    def __init__(self, observation_space, action_space, model_config=None):
        super().__init__()
        cfg = dict(model_config or {})
        d = int(np.prod(observation_space.shape)) + int(np.prod(action_space.shape))
        hid = cfg.get("fcnet_hiddens", [256, 256])
        act = cfg.get("fcnet_activation", "relu")
        self.q1 = nn.Sequential(MLP(d, hid, act), nn.Linear(hid[-1], 1))
        self.q2 = nn.Sequential(MLP(d, hid, act), nn.Linear(hid[-1], 1))

    def forward(self, obs, act):
        x = torch.cat([obs.reshape(obs.shape[0], -1).float(),
                       act.reshape(act.shape[0], -1).float()], -1)
        return self.q1(x).squeeze(-1), self.q2(x).squeeze(-1)


F  # noqa: B018
