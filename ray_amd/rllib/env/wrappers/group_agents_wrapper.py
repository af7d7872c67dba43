"""``GroupAgentsWrapper`` (reference: python/ray/rllib/env/wrappers/group_agents_wrapper.py):
present groups of agents of a MultiAgentEnv as single agents with Tuple spaces (e.g. for
centralized-critic / QMIX-style training). A group's observation and action are tuples
in the group's agent order; its reward is the sum of its members' rewards; it is done
when all its members are."""

from __future__ import annotations

from typing import Dict, List

from ray_amd.rllib.env.multi_agent_env import MultiAgentEnv

GROUP_REWARDS = "_group_rewards"
GROUP_INFO = "_group_info"


class GroupAgentsWrapper(MultiAgentEnv):
    def __init__(self, env, groups: Dict[str, List], obs_space=None, act_space=None):
        self.env = env
        self.groups = {g: list(a) for g, a in groups.items()}
        self.agent_id_to_group = {a: g for g, ags in self.groups.items() for a in ags}
        self.possible_agents = list(self.groups) + [
            a for a in (getattr(env, "possible_agents", None) or [])
            if a not in self.agent_id_to_group]
        self.agents = list(self.possible_agents)
        if obs_space is not None:
            self.observation_space = obs_space
        if act_space is not None:
            self.action_space = act_space
        self.observation_spaces = {g: obs_space for g in self.groups} if obs_space else None
        self.action_spaces = {g: act_space for g in self.groups} if act_space else None

    def reset(self, *, seed=None, options=None):
        obs, info = self.env.reset(seed=seed, options=options)
        return self._group_items(obs), self._group_items(info, agg=lambda v: v)

    def step(self, action_dict):
        actions = {}
        for k, v in action_dict.items():
            if k in self.groups:
                for a, x in zip(self.groups[k], v):
                    actions[a] = x
            else:
                actions[k] = v
        obs, rew, term, trunc, info = self.env.step(actions)
        obs = self._group_items(obs)
        grouped_rew = self._group_items(rew, agg=lambda v: sum(x for x in v if x is not None))
        term = self._group_items(term, agg=all)
        trunc = self._group_items(trunc, agg=all)
        info = self._group_items(info, agg=lambda v: {GROUP_INFO: list(v)})
        for g in self.groups:  # the members' individual rewards, for reference
            if g in grouped_rew and isinstance(info.get(g), dict):
                info[g][GROUP_REWARDS] = [rew.get(a) for a in self.groups[g]]
        term["__all__"] = bool(term.get("__all__", False)) or all(
            term.get(g, False) for g in self.groups)
        trunc["__all__"] = bool(trunc.get("__all__", False))
        return obs, grouped_rew, term, trunc, info

    def _group_items(self, items: dict, agg=tuple):
        out = {}
        for g, ags in self.groups.items():
            vals = [items.get(a) for a in ags]
            present = [v for v in vals if v is not None] if agg is not tuple else vals
            if any(a in items for a in ags):
                out[g] = agg(present) if agg is not tuple else tuple(vals)
        for k, v in items.items():
            if k not in self.agent_id_to_group:
                out[k] = v
        return out
