"""ray_amd.rllib — reinforcement learning on MI355X (reference: rllib/)."""
from ray_amd.rllib.env.envs import register_env  # noqa: F401
from ray_amd.rllib.env.envs import Env  # noqa: F401,E402
from ray_amd.rllib.env.multi_agent_env import MultiAgentEnv  # noqa: F401,E402
from ray_amd.rllib.policy_sample_batch import (DEFAULT_POLICY_ID,  # noqa: F401,E402
                                               MultiAgentBatch, SampleBatch, concat_samples)
from ray_amd.rllib.env.env_runner import SingleAgentEnvRunner  # noqa: F401,E402

from ray_amd.rllib.env.external_env import ExternalEnv  # noqa: F401,E402
from ray_amd.rllib.env.vector_env import VectorEnv  # noqa: F401,E402
from ray_amd.rllib.policy import Policy, TFPolicy, TorchPolicy  # noqa: F401,E402

# classic-stack names: the env runner is this stack's rollout worker
RolloutWorker = SingleAgentEnvRunner
BaseEnv = Env
