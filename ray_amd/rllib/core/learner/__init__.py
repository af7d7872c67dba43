"""``ray.rllib.core.learner`` (reference: python/ray/rllib/core/learner/): the torch
``Learner`` (loss, HIP-graph-captured SGD step, module / state API) in ``learner.py``,
``LearnerGroup`` in ``learner_group.py``, ``TorchLearner`` in ``torch/torch_learner.py``."""

from ray_amd.rllib.core.learner.learner import (  # noqa: F401
    DEFAULT_MODULE_ID, APPOTorchLearner, Fragments, IMPALATorchLearner, Learner,
    LearnerActor, LearnerGroup, MultiAgentLearnerGroup, PPOTorchLearner, TorchLearner,
    _learner_call, _learner_call_kw, _learner_cls, concat_batches, pad_fragment)

__all__ = ["Learner", "LearnerGroup", "MultiAgentLearnerGroup", "TorchLearner"]
