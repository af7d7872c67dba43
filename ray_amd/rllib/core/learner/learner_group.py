"""``ray.rllib.core.learner.learner_group`` (reference path): ``LearnerGroup`` (local
learner or learner actors in one RCCL group), defined with the Learner."""

from ray_amd.rllib.core.learner.learner import LearnerGroup, MultiAgentLearnerGroup  # noqa
