"""Old-stack evaluation helpers (reference: rllib/evaluation/)."""

from ray_amd.rllib.evaluation.postprocessing import (Postprocessing,  # noqa: F401
                                                     compute_advantages,
                                                     compute_gae_for_sample_batch,
                                                     discount_cumsum)
from ray_amd.rllib.evaluation.metrics import (collect_episodes, collect_metrics,  # noqa: F401
                                              summarize_episodes)
from ray_amd.rllib.evaluation.sample_batch_builder import (  # noqa: F401
    MultiAgentSampleBatchBuilder, SampleBatchBuilder)
from ray_amd.rllib.env.env_runner import SingleAgentEnvRunner as RolloutWorker  # noqa: F401
from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode as Episode  # noqa: F401
from ray_amd.rllib.policy_sample_batch import MultiAgentBatch, SampleBatch  # noqa: F401


class SyncSampler:
    """The reference's synchronous sampler over one worker: ``get_data()`` is one
    ``sample()`` of the env runner (old-stack code path)."""

    def __init__(self, *, worker=None, env=None, clip_rewards=None, rollout_fragment_length=None,
                 **kw):
        self.worker = worker
        self.rollout_fragment_length = rollout_fragment_length

    def get_data(self):
        return self.worker.sample(self.rollout_fragment_length)

    def get_metrics(self):
        return [self.worker.get_metrics()]
