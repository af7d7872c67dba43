"""Multi-agent env API (reference: rllib/env/multi_agent_env.py: MultiAgentEnv,
make_multi_agent; rllib/examples/envs/classes/multi_agent.py: MultiAgentCartPole;
turn-based examples: TurnBasedGuess (delayed-credit probe) and TicTacToe).

``reset() -> (obs_dict, info_dict)``; ``step(action_dict) -> (obs, rewards, terminateds,
truncateds, infos)`` with per-agent dicts and the ``"__all__"`` key in ``terminateds`` /
``truncateds`` marking the end of the whole episode."""

from __future__ import annotations

import numpy as np

from ray_amd.rllib.env import spaces
from ray_amd.rllib.env.envs import Env, make_env, register_env


class MultiAgentEnv(Env):
    observation_spaces: dict = None
    action_spaces: dict = None
    possible_agents: list = None
    agents: list = None

    def get_agent_ids(self):
        return set(self.possible_agents or self.agents or [])

    def get_observation_space(self, agent_id):
        if self.observation_spaces:
            return self.observation_spaces[agent_id]
        return self.observation_space

    def get_action_space(self, agent_id):
        if self.action_spaces:
            return self.action_spaces[agent_id]
        return self.action_space

    def observation_space_contains(self, x: dict) -> bool:
        return all(self.get_observation_space(a).contains(v) for a, v in x.items())

    def action_space_contains(self, x: dict) -> bool:
        return all(self.get_action_space(a).contains(v) for a, v in x.items())

    def action_space_sample(self, agent_ids=None) -> dict:
        ids = agent_ids if agent_ids is not None else sorted(self.get_agent_ids(), key=str)
        return {a: self.get_action_space(a).sample() for a in ids}

    def observation_space_sample(self, agent_ids=None) -> dict:
        ids = agent_ids if agent_ids is not None else sorted(self.get_agent_ids(), key=str)
        return {a: self.get_observation_space(a).sample() for a in ids}

    def with_agent_groups(self, groups: dict, obs_space=None, act_space=None):
        """This env with agent groups presented as single agents (GroupAgentsWrapper)."""
        from ray_amd.rllib.env.wrappers.group_agents_wrapper import GroupAgentsWrapper

        return GroupAgentsWrapper(self, groups, obs_space, act_space)

    def to_base_env(self, make_env=None, num_envs: int = 1, remote_envs: bool = False,
                    **kw):
        from ray_amd.rllib.env.base_env import convert_to_base_env

        return convert_to_base_env(self, make_env=make_env, num_envs=num_envs,
                                   remote_envs=remote_envs)


def make_multi_agent(env_name_or_creator):
    """Wrap a single-agent env into a MultiAgentEnv of ``num_agents`` independent copies
    (env_config["num_agents"]); agent ids are 0..num_agents-1.  An agent that finishes
    drops out; ``__all__`` ends the episode when every copy is done."""

    class _MultiEnv(MultiAgentEnv):
        def __init__(self, config=None):
            cfg = dict(config or {})
            num = int(cfg.pop("num_agents", 1))
            base_seed = cfg.pop("seed", 0) or 0
            self.envs = [make_env(env_name_or_creator, dict(cfg, seed=base_seed * 97 + i))
                         for i in range(num)]
            self.possible_agents = list(range(num))
            self.agents = list(self.possible_agents)
            self.observation_space = self.envs[0].observation_space
            self.action_space = self.envs[0].action_space
            self.observation_spaces = {i: e.observation_space for i, e in enumerate(self.envs)}
            self.action_spaces = {i: e.action_space for i, e in enumerate(self.envs)}
            self._done = set()

        def reset(self, *, seed=None, options=None):
            self._done = set()
            self.agents = list(self.possible_agents)
            obs, infos = {}, {}
            for i, e in enumerate(self.envs):
                obs[i], infos[i] = e.reset(seed=None if seed is None else seed * 97 + i,
                                           options=options)
            return obs, infos

        def step(self, action_dict):
            obs, rew, term, trunc, infos = {}, {}, {}, {}, {}
            for i, a in action_dict.items():
                obs[i], rew[i], term[i], trunc[i], infos[i] = self.envs[i].step(a)
                if term[i] or trunc[i]:
                    self._done.add(i)
            self.agents = [i for i in self.possible_agents if i not in self._done]
            term["__all__"] = len(self._done) == len(self.envs)
            trunc["__all__"] = False
            return obs, rew, term, trunc, infos

        def close(self):
            for e in self.envs:
                e.close()

    _MultiEnv.__name__ = f"MultiAgent{getattr(env_name_or_creator, '__name__', env_name_or_creator)}"
    return _MultiEnv


MultiAgentCartPole = make_multi_agent("CartPole-v1")
MultiAgentPendulum = make_multi_agent("Pendulum-v1")
register_env("MultiAgentCartPole", lambda cfg: MultiAgentCartPole(cfg))
register_env("multi_agent_cartpole", lambda cfg: MultiAgentCartPole(cfg))
register_env("MultiAgentPendulum", lambda cfg: MultiAgentPendulum(cfg))


class TurnBasedGuess(MultiAgentEnv):
    """Two players move in turns. The mover observes a one-hot cue (``num_cues`` wide) and
    earns +1 when its action equals the cue, but the reward is paid only in the step the
    OTHER player answers (the final mover is paid when the episode ends), so a learner
    only improves if rewards are credited to the right, earlier action. An episode is
    ``episode_len`` moves in total (env_config)."""

    def __init__(self, config=None):
        cfg = dict(config or {})
        self.n = int(cfg.get("num_cues", 4))
        self.length = int(cfg.get("episode_len", 10))
        self.rng = np.random.default_rng(cfg.get("seed", 0))
        self.possible_agents = ["p1", "p2"]
        self.agents = list(self.possible_agents)
        self.observation_space = spaces.Box(0.0, 1.0, (self.n,), np.float32)
        self.action_space = spaces.Discrete(self.n)

    def _cue(self):
        self.target = int(self.rng.integers(self.n))
        o = np.zeros(self.n, np.float32)
        o[self.target] = 1.0
        return o

    def reset(self, *, seed=None, options=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.t = 0
        self.mover = "p1"
        self.owed = None  # (player, reward) not yet paid
        return {"p1": self._cue()}, {}

    def step(self, action_dict):
        a = int(action_dict[self.mover])
        earned = 1.0 if a == self.target else 0.0
        rew = {}
        if self.owed is not None:
            rew[self.owed[0]] = self.owed[1]
        self.owed = (self.mover, earned)
        self.t += 1
        done = self.t >= self.length
        if done:
            rew[self.mover] = rew.get(self.mover, 0.0) + earned
            term = {"__all__": True, "p1": True, "p2": True}
            return {}, rew, term, {"__all__": False}, {}
        self.mover = "p2" if self.mover == "p1" else "p1"
        return {self.mover: self._cue()}, rew, {"__all__": False}, {"__all__": False}, {}


class TicTacToe(MultiAgentEnv):
    """Turn-based 3x3 tic-tac-toe between ``player1`` (moves first) and ``player2``
    (reference: rllib/examples/envs/classes/multi_agent/tic_tac_toe.py). Observation: the
    board from the mover's view (+1 own, -1 opponent, 0 empty; 9 floats); action: a cell.
    A win pays +1 / -1; an illegal move (occupied cell) ends the game with -1 for the mover
    (+0 for the other); a full board is a draw (0, 0)."""

    LINES = ((0, 1, 2), (3, 4, 5), (6, 7, 8), (0, 3, 6), (1, 4, 7), (2, 5, 8), (0, 4, 8),
             (2, 4, 6))

    def __init__(self, config=None):
        self.possible_agents = ["player1", "player2"]
        self.agents = list(self.possible_agents)
        self.observation_space = spaces.Box(-1.0, 1.0, (9,), np.float32)
        self.action_space = spaces.Discrete(9)

    def _obs(self, who):
        sign = 1.0 if who == "player1" else -1.0
        return (self.board * sign).astype(np.float32)

    def reset(self, *, seed=None, options=None):
        self.board = np.zeros(9, np.float32)  # +1 player1, -1 player2
        self.mover = "player1"
        return {self.mover: self._obs(self.mover)}, {}

    def step(self, action_dict):
        who = self.mover
        other = "player2" if who == "player1" else "player1"
        cell = int(action_dict[who])
        done = {"__all__": True, "player1": True, "player2": True}
        if self.board[cell] != 0:
            return {}, {who: -1.0, other: 0.0}, done, {"__all__": False}, {}
        self.board[cell] = 1.0 if who == "player1" else -1.0
        v = self.board[cell]
        if any(all(self.board[i] == v for i in ln) for ln in self.LINES):
            return {}, {who: 1.0, other: -1.0}, done, {"__all__": False}, {}
        if not (self.board == 0).any():
            return {}, {who: 0.0, other: 0.0}, done, {"__all__": False}, {}
        self.mover = other
        return {other: self._obs(other)}, {}, {"__all__": False}, {"__all__": False}, {}


register_env("TurnBasedGuess", lambda cfg: TurnBasedGuess(cfg))
register_env("TicTacToe", lambda cfg: TicTacToe(cfg))
