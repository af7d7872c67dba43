"""Off-policy estimators (reference: rllib/offline/estimators/__init__.py)."""

from .direct_method import DirectMethod, DoublyRobust
from .fqe_torch_model import FQETorchModel
from .importance_sampling import ImportanceSampling, WeightedImportanceSampling
from .off_policy_estimator import OfflineEvaluator, OffPolicyEstimator, split_by_episode

__all__ = ["DirectMethod", "DoublyRobust", "FQETorchModel", "ImportanceSampling",
           "OfflineEvaluator", "OffPolicyEstimator", "WeightedImportanceSampling",
           "split_by_episode"]
