"""``ray.rllib.algorithms.sac`` (reference: python/ray/rllib/algorithms/sac/):
the algorithm and its config in ``sac.py``, the learner in ``sac_learner.py`` /
``torch/sac_torch_learner.py``."""

from ray_amd.rllib.algorithms.sac.sac import SAC, SACConfig  # noqa: F401
from ray_amd.rllib.algorithms.sac.sac_learner import SACLearner  # noqa: F401

from ray_amd.rllib.algorithms.sac.sac import _SACModule  # noqa: F401

__all__ = ['SAC', 'SACConfig', 'SACLearner']
