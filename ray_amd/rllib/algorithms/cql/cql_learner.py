"""``CQLLearner`` (reference: python/ray/rllib/algorithms/cql/cql_learner.py)."""

from ray_amd.rllib.algorithms.cql.cql import CQLLearner as CQLLearner  # noqa: F401
