"""``ray.rllib.algorithms.cql`` (reference: python/ray/rllib/algorithms/cql/):
the algorithm and its config in ``cql.py``, the learner in ``cql_learner.py`` /
``torch/cql_torch_learner.py``."""

from ray_amd.rllib.algorithms.cql.cql import CQL, CQLConfig  # noqa: F401
from ray_amd.rllib.algorithms.cql.cql_learner import CQLLearner  # noqa: F401

__all__ = ['CQL', 'CQLConfig', 'CQLLearner']
