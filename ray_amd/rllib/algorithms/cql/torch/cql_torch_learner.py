"""``CQLTorchLearner`` (reference: python/ray/rllib/algorithms/cql/torch/cql_torch_learner.py):
ray_amd's learners are torch learners; this is ``CQLLearner``."""

from ray_amd.rllib.algorithms.cql.cql_learner import CQLLearner as CQLTorchLearner  # noqa: F401
