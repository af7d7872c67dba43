"""``ray.rllib.algorithms.impala`` (reference: python/ray/rllib/algorithms/impala/):
the algorithm and its config in ``impala.py``, the learner in ``impala_learner.py`` /
``torch/impala_torch_learner.py``."""

from ray_amd.rllib.algorithms.impala.impala import IMPALA, IMPALAConfig  # noqa: F401
from ray_amd.rllib.algorithms.impala.impala_learner import IMPALALearner  # noqa: F401

from ray_amd.rllib.algorithms.impala.impala import APPO, APPOConfig  # noqa: F401

__all__ = ['IMPALA', 'IMPALAConfig', 'IMPALALearner']
