"""Old-stack exploration strategies (reference: python/ray/rllib/utils/exploration/).

An ``Exploration`` turns an action distribution into the action taken:
``get_exploration_action(action_distribution=..., timestep=..., explore=...)`` returns
``(actions, logp)``. Epsilon and noise scales anneal with ``timestep`` through the
schedules of ``rllib/utils/schedules``; the ``PerWorker*`` variants give each env runner
its own constant scale (Ape-X style: ``eps_i = 0.4 ** (1 + 7 i / (n - 1))``).

New-stack RLModules sample inside ``forward_exploration`` (ray_amd's default modules draw
with Gumbel-max / Gaussian noise on device); these classes serve old-stack policies."""

from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from ray_amd.rllib.utils.schedules import ConstantSchedule, PiecewiseSchedule


def _schedule(initial, final, timesteps):
    return PiecewiseSchedule([(0, initial), (int(timesteps), final)],
                             outside_value=final)


def _value(s, t):
    return s.value(t) if hasattr(s, "value") else s(t)


def _dist_parts(dist):
    """(kind, tensor): 'categorical' logits or 'gaussian' mean for ray_amd's and the
    reference-style distribution objects alike."""
    inputs = getattr(dist, "inputs", dist)
    if not isinstance(inputs, torch.Tensor):
        inputs = torch.as_tensor(np.asarray(inputs), dtype=torch.float32)
    name = type(dist).__name__.lower()
    if "gaussian" in name or "deterministic" in name:
        mean = getattr(dist, "mean", None)
        return "gaussian", mean if mean is not None else inputs
    return "categorical", inputs


class Exploration:
    def __init__(self, action_space=None, *, framework: str = "torch", policy_config=None,
                 model=None, num_workers: int = 0, worker_index: int = 0, **kw):
        self.action_space = action_space
        self.policy_config = policy_config or {}
        self.model = model
        self.num_workers = num_workers
        self.worker_index = worker_index
        self.last_timestep = 0

    def before_compute_actions(self, *, timestep=None, explore=None, **kw):
        pass

    def get_exploration_action(self, *, action_distribution, timestep, explore: bool = True):
        raise NotImplementedError

    def on_episode_start(self, *a, **k):
        pass

    def on_episode_end(self, *a, **k):
        pass

    def postprocess_trajectory(self, policy, sample_batch, tf_sess=None):
        return sample_batch

    def get_state(self, sess=None) -> dict:
        return {"last_timestep": self.last_timestep}

    def set_state(self, state: dict, sess=None) -> None:
        self.last_timestep = state.get("last_timestep", 0)

    def get_exploration_optimizer(self, optimizers):
        return optimizers


class StochasticSampling(Exploration):
    """Sample from the distribution when exploring, its mode otherwise (optionally
    uniform random actions for the first ``random_timesteps``)."""

    def __init__(self, action_space=None, *, random_timesteps: int = 0, **kw):
        super().__init__(action_space, **kw)
        self.random_timesteps = random_timesteps

    def get_exploration_action(self, *, action_distribution, timestep=None, explore=True):
        self.last_timestep = timestep if timestep is not None else self.last_timestep + 1
        if explore and self.last_timestep < self.random_timesteps and \
                self.action_space is not None:
            n = _batch(action_distribution)
            a = torch.as_tensor(np.stack([self.action_space.sample() for _ in range(n)]))
            return a, torch.zeros(n)
        if explore:
            a = action_distribution.sample()
            return a, action_distribution.sampled_action_logp()
        return action_distribution.deterministic_sample(), torch.zeros(_batch(
            action_distribution))


def _batch(dist) -> int:
    inputs = getattr(dist, "inputs", None)
    return int(inputs.shape[0]) if inputs is not None else 1


class Random(Exploration):
    def get_exploration_action(self, *, action_distribution, timestep=None, explore=True):
        n = _batch(action_distribution)
        if explore:
            a = torch.as_tensor(np.stack([self.action_space.sample() for _ in range(n)]))
        else:
            a = action_distribution.deterministic_sample()
        return a, torch.zeros(n)


class EpsilonGreedy(Exploration):
    def __init__(self, action_space=None, *, initial_epsilon: float = 1.0,
                 final_epsilon: float = 0.05, warmup_timesteps: int = 0,
                 epsilon_timesteps: int = int(1e5), epsilon_schedule=None, **kw):
        super().__init__(action_space, **kw)
        self.epsilon_schedule = epsilon_schedule or PiecewiseSchedule(
            [(0, initial_epsilon), (warmup_timesteps, initial_epsilon),
             (warmup_timesteps + epsilon_timesteps, final_epsilon)],
            outside_value=final_epsilon)
        self._rng = np.random.default_rng(kw.get("seed"))

    def epsilon(self, timestep) -> float:
        return float(_value(self.epsilon_schedule, timestep))

    def get_exploration_action(self, *, action_distribution, timestep=None, explore=True):
        self.last_timestep = timestep if timestep is not None else self.last_timestep + 1
        kind, q = _dist_parts(action_distribution)
        greedy = q.argmax(-1)
        if not explore:
            return greedy, torch.zeros(len(greedy))
        eps = self.epsilon(self.last_timestep)
        n, na = q.shape[0], q.shape[-1]
        rand = torch.as_tensor(self._rng.integers(0, na, n))
        take = torch.as_tensor(self._rng.random(n) < eps)
        return torch.where(take, rand, greedy), torch.zeros(n)

    def get_state(self, sess=None):
        return {"last_timestep": self.last_timestep,
                "cur_epsilon": self.epsilon(self.last_timestep)}


def _per_worker_scale(base: float, exponent: float, worker_index: int, num_workers: int):
    if num_workers <= 0:
        return 0.0 if worker_index == 0 else base
    if worker_index == 0:
        return 0.0  # the local (evaluation-style) worker acts greedily
    return base ** (1 + (worker_index - 1) / max(1, num_workers - 1) * exponent)


class PerWorkerEpsilonGreedy(EpsilonGreedy):
    def __init__(self, action_space=None, *, num_workers: int = 0, worker_index: int = 0,
                 **kw):
        eps = _per_worker_scale(0.4, 7.0, worker_index, num_workers)
        kw["epsilon_schedule"] = ConstantSchedule(eps)
        super().__init__(action_space, num_workers=num_workers, worker_index=worker_index,
                         **kw)


class SoftQ(StochasticSampling):
    """Boltzmann exploration: sample from softmax(Q / temperature)."""

    def __init__(self, action_space=None, *, temperature: float = 1.0, **kw):
        super().__init__(action_space, **kw)
        self.temperature = temperature

    def get_exploration_action(self, *, action_distribution, timestep=None, explore=True):
        _, q = _dist_parts(action_distribution)
        if not explore:
            return q.argmax(-1), torch.zeros(q.shape[0])
        d = torch.distributions.Categorical(logits=q / self.temperature)
        a = d.sample()
        return a, d.log_prob(a)


class GaussianNoise(Exploration):
    """Deterministic action + N(0, stddev * scale(t)) noise, uniform random actions for
    the first ``random_timesteps``; clipped to the action space."""

    def __init__(self, action_space=None, *, random_timesteps: int = 1000,
                 stddev: float = 0.1, initial_scale: float = 1.0, final_scale: float = 0.02,
                 scale_timesteps: int = 10000, scale_schedule=None, **kw):
        super().__init__(action_space, **kw)
        self.random_timesteps = random_timesteps
        self.stddev = stddev
        self.scale_schedule = scale_schedule or _schedule(initial_scale, final_scale,
                                                          scale_timesteps)
        self._rng = np.random.default_rng(kw.get("seed"))

    def _noise(self, shape):
        return torch.as_tensor(self._rng.normal(0.0, self.stddev, shape), dtype=torch.float32)

    def get_exploration_action(self, *, action_distribution, timestep=None, explore=True):
        self.last_timestep = timestep if timestep is not None else self.last_timestep + 1
        det = action_distribution.deterministic_sample()
        n = det.shape[0]
        if not explore:
            return det, torch.zeros(n)
        if self.last_timestep < self.random_timesteps:
            a = torch.as_tensor(np.stack([self.action_space.sample() for _ in range(n)]),
                                dtype=torch.float32)
        else:
            a = det + float(_value(self.scale_schedule, self.last_timestep)) * \
                self._noise(tuple(det.shape))
        if self.action_space is not None and hasattr(self.action_space, "low"):
            a = torch.clamp(a, torch.tensor(np.array(self.action_space.low)),
                            torch.tensor(np.array(self.action_space.high)))
        return a, torch.zeros(n)


class PerWorkerGaussianNoise(GaussianNoise):
    def __init__(self, action_space=None, *, num_workers: int = 0, worker_index: int = 0,
                 **kw):
        scale = _per_worker_scale(0.4, 7.0, worker_index, num_workers)
        kw["scale_schedule"] = ConstantSchedule(scale)
        super().__init__(action_space, num_workers=num_workers, worker_index=worker_index,
                         **kw)


class OrnsteinUhlenbeckNoise(GaussianNoise):
    """Temporally correlated noise: x += theta * (-x) + sigma * N(0, 1), scaled."""

    def __init__(self, action_space=None, *, ou_theta: float = 0.15, ou_sigma: float = 0.2,
                 ou_base_scale: float = 0.1, **kw):
        super().__init__(action_space, **kw)
        self.ou_theta, self.ou_sigma, self.ou_base_scale = ou_theta, ou_sigma, ou_base_scale
        self.ou_state = None

    def _noise(self, shape):
        if self.ou_state is None or self.ou_state.shape != shape:
            self.ou_state = np.zeros(shape)
        self.ou_state = self.ou_state + self.ou_theta * (-self.ou_state) + \
            self.ou_sigma * self._rng.normal(size=shape)
        rng = (self.action_space.high - self.action_space.low) \
            if self.action_space is not None and hasattr(self.action_space, "high") else 1.0
        return torch.as_tensor(self.ou_base_scale * self.ou_state * rng, dtype=torch.float32)

    def get_state(self, sess=None):
        return {"last_timestep": self.last_timestep, "ou_state": self.ou_state}

    def set_state(self, state, sess=None):
        super().set_state(state)
        self.ou_state = state.get("ou_state")


class PerWorkerOrnsteinUhlenbeckNoise(OrnsteinUhlenbeckNoise):
    def __init__(self, action_space=None, *, num_workers: int = 0, worker_index: int = 0,
                 **kw):
        scale = _per_worker_scale(0.4, 7.0, worker_index, num_workers)
        kw["scale_schedule"] = ConstantSchedule(scale)
        super().__init__(action_space, num_workers=num_workers, worker_index=worker_index,
                         **kw)


class ParameterNoise(Exploration):
    """Perturb the model's weights with N(0, sigma) for a whole episode (Plappert et al.
    2018): ``on_episode_start`` adds fresh noise, ``on_episode_end`` removes it; actions
    come from the perturbed model's mode."""

    def __init__(self, action_space=None, *, initial_stddev: float = 1.0, **kw):
        super().__init__(action_space, **kw)
        self.stddev = initial_stddev
        self._noise = None

    def on_episode_start(self, policy=None, *, environment=None, episode=None, tf_sess=None,
                         **kw):
        model = self.model if self.model is not None else getattr(policy, "model", None)
        if model is None:
            return
        with torch.no_grad():
            self._noise = [torch.randn_like(p) * self.stddev for p in model.parameters()]
            for p, n in zip(model.parameters(), self._noise):
                p.add_(n)

    def on_episode_end(self, policy=None, *, environment=None, episode=None, tf_sess=None,
                       **kw):
        model = self.model if self.model is not None else getattr(policy, "model", None)
        if model is None or self._noise is None:
            return
        with torch.no_grad():
            for p, n in zip(model.parameters(), self._noise):
                p.sub_(n)
        self._noise = None

    def get_exploration_action(self, *, action_distribution, timestep=None, explore=True):
        return action_distribution.deterministic_sample(), torch.zeros(
            _batch(action_distribution))


__all__ = ["Exploration", "EpsilonGreedy", "GaussianNoise", "OrnsteinUhlenbeckNoise",
           "ParameterNoise", "PerWorkerEpsilonGreedy", "PerWorkerGaussianNoise",
           "PerWorkerOrnsteinUhlenbeckNoise", "Random", "SoftQ", "StochasticSampling"]
