"""Built-in environments + registry (reference: rllib/env/*, ray.tune.registry.register_env).

gymnasium is not installed, so the classic-control envs used by the reference's
tests/tuned examples are re-implemented from their published dynamics, plus a
synthetic Atari env with the exact Atari observation/action shapes used by the
PPO/IMPALA Atari benchmarks (84x84x4 uint8 frames, Discrete(6))."""

from __future__ import annotations

import math

import numpy as np

from ray_amd.rllib.env import spaces

_REGISTRY: dict = {}


class Env:
    """gymnasium.Env-compatible interface: reset(seed) -> (obs, info);
    step(a) -> (obs, reward, terminated, truncated, info)."""

    observation_space: spaces.Space = None
    action_space: spaces.Space = None
    metadata = {}
    spec = None

    def reset(self, *, seed=None, options=None):
        raise NotImplementedError

    def step(self, action):
        raise NotImplementedError

    def close(self):
        pass

    def render(self):
        return None

    @property
    def unwrapped(self):
        return self


def register_env(name: str, creator):
    _REGISTRY[name] = creator


def _wrap(e):
    """ExternalEnvs are stepped through their gym-style adapter."""
    from ray_amd.rllib.env.external_env import ExternalEnv, ExternalEnvAdapter

    return ExternalEnvAdapter(e) if isinstance(e, ExternalEnv) else e


def make_env(env, env_config=None):
    from ray_amd.rllib.env.env_context import EnvContext

    # creators get an EnvContext (a dict with worker_index / vector_index / num_workers)
    cfg = env_config if isinstance(env_config, EnvContext) else EnvContext(env_config or {})
    if isinstance(env, str):
        if env in _REGISTRY:
            return _wrap(_REGISTRY[env](cfg))
        raise ValueError(f"unknown env {env!r}; registered: {sorted(_REGISTRY)}")
    if isinstance(env, type):
        try:
            return _wrap(env(cfg))
        except TypeError:
            return _wrap(env())
    if callable(env):
        return _wrap(env(cfg))
    raise ValueError(f"cannot build env from {env!r}")


class CartPoleEnv(Env):
    """CartPole-v1 dynamics (Barto, Sutton & Anderson 1983; gymnasium classic_control)."""

    def __init__(self, config=None):
        self.gravity, self.masscart, self.masspole = 9.8, 1.0, 0.1
        self.total_mass = self.masspole + self.masscart
        self.length = 0.5
        self.polemass_length = self.masspole * self.length
        self.force_mag, self.tau = 10.0, 0.02
        self.theta_threshold = 12 * 2 * math.pi / 360
        self.x_threshold = 2.4
        self.max_steps = int((config or {}).get("max_episode_steps", 500))
        high = np.array([self.x_threshold * 2, np.inf, self.theta_threshold * 2, np.inf],
                        dtype=np.float32)
        self.observation_space = spaces.Box(-high, high, dtype=np.float32)
        self.action_space = spaces.Discrete(2)
        self.rng = np.random.default_rng()
        self.state = None
        self.t = 0

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.state = self.rng.uniform(-0.05, 0.05, size=4)
        self.t = 0
        return self.state.astype(np.float32), {}

    def step(self, action):
        x, x_dot, th, th_dot = self.state
        force = self.force_mag if action == 1 else -self.force_mag
        ct, st = math.cos(th), math.sin(th)
        temp = (force + self.polemass_length * th_dot ** 2 * st) / self.total_mass
        thacc = (self.gravity * st - ct * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * ct ** 2 / self.total_mass))
        xacc = temp - self.polemass_length * thacc * ct / self.total_mass
        x += self.tau * x_dot
        x_dot += self.tau * xacc
        th += self.tau * th_dot
        th_dot += self.tau * thacc
        self.state = np.array([x, x_dot, th, th_dot])
        self.t += 1
        term = bool(x < -self.x_threshold or x > self.x_threshold or th < -self.theta_threshold
                    or th > self.theta_threshold)
        trunc = self.t >= self.max_steps
        return self.state.astype(np.float32), 1.0, term, trunc, {}


class PendulumEnv(Env):
    """Pendulum-v1 dynamics (gymnasium classic_control)."""

    def __init__(self, config=None):
        self.max_speed, self.max_torque, self.dt = 8.0, 2.0, 0.05
        self.g, self.m, self.l = 10.0, 1.0, 1.0
        high = np.array([1.0, 1.0, self.max_speed], dtype=np.float32)
        self.observation_space = spaces.Box(-high, high, dtype=np.float32)
        self.action_space = spaces.Box(-self.max_torque, self.max_torque, shape=(1,),
                                       dtype=np.float32)
        self.rng = np.random.default_rng()
        self.t = 0

    def _obs(self):
        th, thd = self.state
        return np.array([math.cos(th), math.sin(th), thd], dtype=np.float32)

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.state = self.rng.uniform([-math.pi, -1.0], [math.pi, 1.0])
        self.t = 0
        return self._obs(), {}

    def step(self, u):
        th, thd = self.state
        u = float(np.clip(np.asarray(u).reshape(-1)[0], -self.max_torque, self.max_torque))
        ang = ((th + math.pi) % (2 * math.pi)) - math.pi
        cost = ang ** 2 + 0.1 * thd ** 2 + 0.001 * u ** 2
        thd = thd + (3 * self.g / (2 * self.l) * math.sin(th) + 3.0 / (self.m * self.l ** 2) * u
                     ) * self.dt
        thd = float(np.clip(thd, -self.max_speed, self.max_speed))
        th = th + thd * self.dt
        self.state = np.array([th, thd])
        self.t += 1
        return self._obs(), -cost, False, self.t >= 200, {}


class SyntheticAtariEnv(Env):
    """Atari-shaped synthetic env: 84x84x4 uint8 frame stacks, Discrete(6) actions.

    Frames come from a fixed random bank (so per-step cost is a view + small RNG
    draw, like an ALE step + frame-stack wrapper) and reward/termination are
    random with the statistics of Pong-style episodes. Used for throughput
    benchmarks of the PPO / IMPALA Atari configs."""

    def __init__(self, config=None):
        cfg = config or {}
        self.H = self.W = int(cfg.get("dim", 84))
        self.stack = int(cfg.get("framestack", 4))
        self.n_actions = int(cfg.get("num_actions", 6))
        self.episode_len = int(cfg.get("episode_len", 1000))
        self.observation_space = spaces.Box(0, 255, shape=(self.H, self.W, self.stack),
                                            dtype=np.uint8)
        self.action_space = spaces.Discrete(self.n_actions)
        seed = int(cfg.get("seed", 0))
        bank_rng = np.random.default_rng(1234 + seed)
        self.bank = bank_rng.integers(0, 256, size=(64, self.H, self.W, self.stack),
                                      dtype=np.uint8)
        self.rng = np.random.default_rng(seed)
        # per-game reward magnitudes of the stand-ins (Breakout bricks score 1 / 4 / 7,
        # Qbert 25, ...): clip_rewards=True is what maps them to {-1, 0, 1}
        self.reward_values = [float(v) for v in cfg.get("reward_values", (1.0,))]
        self.t = 0
        self.i = 0

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.t = 0
        self.i = int(self.rng.integers(64))
        return self.bank[self.i], {}

    def step(self, action):
        self.t += 1
        self.i = (self.i + 1 + int(action)) & 63
        r = self.rng.random()
        reward = 0.0
        if r < 0.02:
            v = self.reward_values[int(self.rng.integers(len(self.reward_values)))]
            reward = v if r < 0.01 else -v
        term = self.rng.random() < 1.0 / self.episode_len
        return self.bank[self.i], reward, bool(term), self.t >= 10 * self.episode_len, {}


class RandomEnv(Env):
    def __init__(self, config=None):
        cfg = config or {}
        self.observation_space = cfg.get("observation_space", spaces.Box(-1, 1, (4,)))
        self.action_space = cfg.get("action_space", spaces.Discrete(2))
        self.p_done = cfg.get("p_terminated", 0.1)
        self.rng = np.random.default_rng()

    def reset(self, *, seed=None, options=None):
        return self.observation_space.sample(), {}

    def step(self, a):
        return self.observation_space.sample(), float(self.rng.random()), \
            bool(self.rng.random() < self.p_done), False, {}


class RepeatAfterMeEnv(Env):
    """Memory task (reference: rllib/examples/envs/classes/repeat_after_me_env.py): each
    step shows one of ``n`` symbols (one-hot); the reward is +1 for repeating the symbol
    shown ``delay`` steps earlier, -1 otherwise. A memoryless policy averages 0 per step;
    a recurrent one can reach +1."""

    def __init__(self, config=None):
        cfg = config or {}
        self.n = int(cfg.get("num_symbols", 2))
        self.delay = int(cfg.get("repeat_delay", 1))
        self.episode_len = int(cfg.get("episode_len", 20))
        self.observation_space = spaces.Box(0.0, 1.0, (self.n,))
        self.action_space = spaces.Discrete(self.n)
        self.rng = np.random.default_rng(cfg.get("seed"))

    def _obs(self):
        o = np.zeros(self.n, np.float32)
        o[self.hist[-1]] = 1.0
        return o

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.t = 0
        self.hist = [int(self.rng.integers(self.n))]
        return self._obs(), {}

    def step(self, action):
        self.t += 1
        r = 0.0
        if len(self.hist) > self.delay:  # the symbol shown `delay` steps before this one
            r = 1.0 if int(action) == self.hist[-1 - self.delay] else -1.0
        self.hist.append(int(self.rng.integers(self.n)))
        self.hist = self.hist[-(self.delay + 1):]
        return self._obs(), r, False, self.t >= self.episode_len, {}


register_env("CartPole-v1", CartPoleEnv)
register_env("RepeatAfterMeEnv", RepeatAfterMeEnv)
register_env("CartPole-v0", lambda c: CartPoleEnv({"max_episode_steps": 200, **(c or {})}))
register_env("Pendulum-v1", PendulumEnv)
register_env("SyntheticAtari-v0", SyntheticAtariEnv)
# shape-compatible stand-ins for the ALE games of the tuned examples (no ALE in the image)
register_env("ALE/Pong-v5", SyntheticAtariEnv)
for _game, _rv in (("Breakout", (1.0, 4.0, 7.0)), ("BeamRider", (44.0,)), ("Qbert", (25.0,)),
                   ("SpaceInvaders", (5.0, 10.0, 15.0, 30.0))):
    register_env(f"ALE/{_game}-v5",
                 lambda c, _rv=_rv: SyntheticAtariEnv({"reward_values": _rv, **(c or {})}))
register_env("RandomEnv", RandomEnv)
