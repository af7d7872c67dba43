"""``APPOLearner`` (reference: python/ray/rllib/algorithms/appo/appo_learner.py): the shared
torch Learner (core/learner/learner.py) with the APPO loss selected by the config."""

from ray_amd.rllib.core.learner import Learner as APPOLearner  # noqa: F401
