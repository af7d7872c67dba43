"""ConnectorV2 base and pipeline.

API contract (reference: rllib/connectors/connector_v2.py:18 ``ConnectorV2`` —
``__call__(*, rl_module, batch, episodes, explore, shared_data, **kwargs)`` returning
the (possibly new) batch; ``get_state``/``set_state``; ``recompute_output_observation_space``;
connector_pipeline_v2.py ``ConnectorPipelineV2`` with append/prepend/insert_before/
insert_after/remove).

Design: the EnvRunner steps a vector of envs in lock-step, so a connector sees ONE
batched step at a time: ``batch`` is a dict of numpy arrays whose leading dim is the
env index ("obs" before the module, "actions" after it), and ``episodes`` carries the
per-env episode bookkeeping (returns so far, previous action/reward). Stateful
connectors expose their state so the Algorithm can broadcast it with the weights.
"""

from __future__ import annotations


class ConnectorV2:
    """A transformation of a batched env step (or learner batch)."""

    def __init__(self, input_observation_space=None, input_action_space=None, **kwargs):
        self.input_observation_space = input_observation_space
        self.input_action_space = input_action_space

    def __call__(self, *, rl_module=None, batch: dict, episodes=None, explore: bool = True,
                 shared_data: dict | None = None, **kwargs) -> dict:
        raise NotImplementedError

    def recompute_output_observation_space(self, obs_space, act_space):
        return obs_space

    @property
    def observation_space(self):
        return self.recompute_output_observation_space(self.input_observation_space,
                                                       self.input_action_space)

    def get_state(self):
        return {}

    def set_state(self, state):
        pass

    def reset_state(self):
        pass

    def __repr__(self):
        return type(self).__name__


class ConnectorPipelineV2(ConnectorV2):
    def __init__(self, input_observation_space=None, input_action_space=None, connectors=None,
                 **kwargs):
        super().__init__(input_observation_space, input_action_space)
        self.connectors = list(connectors or [])

    def __call__(self, *, rl_module=None, batch: dict, episodes=None, explore: bool = True,
                 shared_data: dict | None = None, **kwargs) -> dict:
        shared = shared_data if shared_data is not None else {}
        for c in self.connectors:
            batch = c(rl_module=rl_module, batch=batch, episodes=episodes, explore=explore,
                      shared_data=shared, **kwargs)
        return batch

    def recompute_output_observation_space(self, obs_space, act_space):
        for c in self.connectors:
            obs_space = c.recompute_output_observation_space(obs_space, act_space)
        return obs_space

    def _index(self, name_or_cls):
        for i, c in enumerate(self.connectors):
            if (isinstance(name_or_cls, str) and type(c).__name__ == name_or_cls) or \
                    (isinstance(name_or_cls, type) and isinstance(c, name_or_cls)):
                return i
        raise ValueError(f"no connector {name_or_cls} in {self.connectors}")

    def append(self, c):
        self.connectors.append(c)

    def prepend(self, c):
        self.connectors.insert(0, c)

    def insert_before(self, name_or_cls, c):
        self.connectors.insert(self._index(name_or_cls), c)

    def insert_after(self, name_or_cls, c):
        self.connectors.insert(self._index(name_or_cls) + 1, c)

    def remove(self, name_or_cls):
        del self.connectors[self._index(name_or_cls)]

    def find(self, cls):
        return [c for c in self.connectors if isinstance(c, cls)]

    def __len__(self):
        return len(self.connectors)

    def get_state(self):
        return {i: c.get_state() for i, c in enumerate(self.connectors)}

    def set_state(self, state):
        for i, c in enumerate(self.connectors):
            if i in state:
                c.set_state(state[i])

    def __repr__(self):
        return f"ConnectorPipelineV2({self.connectors})"


def build_pipeline(factory, obs_space, act_space):
    """config factory (callable(env) or callable(obs, act) -> connector(s)) -> pipeline."""
    if factory is None:
        return ConnectorPipelineV2(obs_space, act_space, [])
    try:
        out = factory(obs_space, act_space)
    except TypeError:
        out = factory(None)
    if isinstance(out, ConnectorPipelineV2):
        return out
    if isinstance(out, ConnectorV2):
        out = [out]
    return ConnectorPipelineV2(obs_space, act_space, list(out or []))
