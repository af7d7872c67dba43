"""Old-stack observation preprocessors (reference: python/ray/rllib/models/preprocessors.py):
``get_preprocessor(space)`` -> a class whose ``transform(obs)`` gives the flat (or image)
array a model consumes: one-hot for Discrete / MultiDiscrete, concatenation for Dict and
Tuple, identity for Box. ray_amd's RLModules take observations unflattened (encoders
flatten on device); these serve old-stack code that preprocesses itself."""

from __future__ import annotations

from typing import Optional

import numpy as np

from ray_amd.rllib.env import spaces


class Preprocessor:
    def __init__(self, obs_space, options: Optional[dict] = None):
        self._obs_space = obs_space
        self._options = options or {}
        self.shape = self._init_shape(obs_space, self._options)
        self._size = int(np.prod(self.shape))

    def _init_shape(self, obs_space, options):
        raise NotImplementedError

    def transform(self, observation) -> np.ndarray:
        raise NotImplementedError

    def write(self, observation, array, offset: int) -> None:
        array[offset:offset + self._size] = self.transform(observation).reshape(-1)

    def check_shape(self, observation) -> None:
        if not self._obs_space.contains(observation):
            raise ValueError(f"observation {observation!r} outside {self._obs_space}")

    @property
    def size(self) -> int:
        return self._size

    @property
    def observation_space(self):
        return spaces.Box(-np.inf, np.inf, self.shape, np.float32)


class NoPreprocessor(Preprocessor):
    def _init_shape(self, obs_space, options):
        return tuple(obs_space.shape)

    def transform(self, observation):
        return np.asarray(observation)

    @property
    def observation_space(self):
        return self._obs_space


class OneHotPreprocessor(Preprocessor):
    def _init_shape(self, obs_space, options):
        if isinstance(obs_space, spaces.MultiDiscrete):
            return (int(np.sum(obs_space.nvec)),)
        return (int(obs_space.n),)

    def transform(self, observation):
        out = np.zeros(self.shape, np.float32)
        if isinstance(self._obs_space, spaces.MultiDiscrete):
            off = 0
            for v, n in zip(np.asarray(observation).reshape(-1), self._obs_space.nvec):
                out[off + int(v)] = 1.0
                off += int(n)
        else:
            out[int(observation)] = 1.0
        return out


class _FlatteningPreprocessor(Preprocessor):
    def _children(self, obs_space):
        raise NotImplementedError

    def _init_shape(self, obs_space, options):
        self.preprocessors = [get_preprocessor(s)(s, options) for s in self._children(obs_space)]
        return (int(sum(p.size for p in self.preprocessors)),)

    def _items(self, observation):
        raise NotImplementedError

    def transform(self, observation):
        out = np.zeros(self.shape, np.float32)
        off = 0
        for p, o in zip(self.preprocessors, self._items(observation)):
            out[off:off + p.size] = np.asarray(p.transform(o), np.float32).reshape(-1)
            off += p.size
        return out


class TupleFlatteningPreprocessor(_FlatteningPreprocessor):
    def _children(self, obs_space):
        return list(obs_space.spaces)

    def _items(self, observation):
        return list(observation)


class DictFlatteningPreprocessor(_FlatteningPreprocessor):
    def _children(self, obs_space):
        return [obs_space.spaces[k] for k in sorted(obs_space.spaces)]

    def _items(self, observation):
        return [observation[k] for k in sorted(self._obs_space.spaces)]


class GenericPixelPreprocessor(Preprocessor):
    """Resize (nearest) to ``dim`` x ``dim``, optional grayscale and [-1, 1] scaling."""

    def _init_shape(self, obs_space, options):
        self._grayscale = options.get("grayscale", False)
        self._zero_mean = options.get("zero_mean", True)
        self._dim = int(options.get("dim", 84))
        return (self._dim, self._dim, 1 if self._grayscale else obs_space.shape[-1])

    def transform(self, observation):
        x = np.asarray(observation, np.float32)
        h, w = x.shape[:2]
        ri = (np.arange(self._dim) * h // self._dim)
        ci = (np.arange(self._dim) * w // self._dim)
        x = x[ri][:, ci]
        if self._grayscale:
            x = x.mean(-1, keepdims=True)
        return (x - 128.0) / 128.0 if self._zero_mean else x / 255.0


def get_preprocessor(space):
    """The preprocessor class for ``space``."""
    if isinstance(space, (spaces.Discrete, spaces.MultiDiscrete)):
        return OneHotPreprocessor
    if isinstance(space, spaces.Tuple):
        return TupleFlatteningPreprocessor
    if isinstance(space, spaces.Dict):
        return DictFlatteningPreprocessor
    return NoPreprocessor
