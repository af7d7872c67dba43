"""``ray.rllib.algorithms.marwil`` (reference: python/ray/rllib/algorithms/marwil/):
the algorithm and its config in ``marwil.py``, the learner in ``marwil_learner.py`` /
``torch/marwil_torch_learner.py``."""

from ray_amd.rllib.algorithms.marwil.marwil import MARWIL, MARWILConfig  # noqa: F401
from ray_amd.rllib.algorithms.marwil.marwil_learner import MARWILLearner  # noqa: F401

from ray_amd.rllib.algorithms.marwil.marwil import BC, BCConfig  # noqa: F401

__all__ = ['MARWIL', 'MARWILConfig', 'MARWILLearner']
