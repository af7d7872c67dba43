"""Multi-agent env API (reference: rllib/env/multi_agent_env.py: MultiAgentEnv,
make_multi_agent; rllib/examples/envs/classes/multi_agent.py: MultiAgentCartPole).

``reset() -> (obs_dict, info_dict)``; ``step(action_dict) -> (obs, rewards, terminateds,
truncateds, infos)`` with per-agent dicts and the ``"__all__"`` key in ``terminateds`` /
``truncateds`` marking the end of the whole episode."""

from __future__ import annotations

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
