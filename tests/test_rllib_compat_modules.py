"""Reference import paths of RLlib's older API surface (round 6): ModelCatalog custom
models running inside PPO (across runner processes), schedules, metric names, check_env,
compute_advantages, synchronous_parallel_sample / train_one_step, the appo / bc packages
and the DeepMind Atari wrappers."""
import numpy as np
import pytest
import torch.nn as nn

import ray_amd as ray
from ray_amd.rllib.models import ModelCatalog
from ray_amd.rllib.models.torch import TorchModelV2


class _TinyModel(TorchModelV2):
    def __init__(self, obs_space, action_space, num_outputs, model_config, name, hidden=16):
        super().__init__(obs_space, action_space, num_outputs, model_config, name)
        d = int(np.prod(obs_space.shape))
        self.body = nn.Sequential(nn.Linear(d, hidden), nn.Tanh())
        self.pi = nn.Linear(hidden, num_outputs)
        self.v = nn.Linear(hidden, 1)
        self._v = None

    def forward(self, input_dict, state, seq_lens):
        h = self.body(input_dict["obs_flat"])
        self._v = self.v(h).squeeze(-1)
        return self.pi(h), state

    def value_function(self):
        return self._v


def test_custom_model_in_ppo_with_remote_runners():
    from ray_amd.rllib.algorithms import PPOConfig
    from ray_amd.rllib.execution import synchronous_parallel_sample, train_one_step

    ModelCatalog.register_custom_model("tiny", _TinyModel)
    ray.init(num_cpus=4)
    try:
        algo = (PPOConfig().environment("CartPole-v1")
                .env_runners(num_env_runners=2, num_envs_per_env_runner=1,
                             rollout_fragment_length=32)
                .training(train_batch_size=64, minibatch_size=32, num_epochs=1,
                          model={"custom_model": "tiny", "custom_model_config": {"hidden": 8}})
                .debugging(seed=0)).build()
        r = algo.train()
        assert r["training_iteration"] == 1
        assert isinstance(algo.get_module().m.model, _TinyModel)
        b = synchronous_parallel_sample(worker_set=algo, max_env_steps=64)
        assert len(b["rewards"]) >= 64 or np.asarray(b["rewards"]).size >= 64
        algo.stop()
    finally:
        ray.shutdown()


def test_schedules_metrics_checks_postprocessing():
    from ray_amd.rllib.env.envs import make_env
    from ray_amd.rllib.evaluation.postprocessing import (Postprocessing, compute_advantages,
                                                         discount_cumsum)
    from ray_amd.rllib.utils.metrics import ENV_RUNNER_RESULTS, EPISODE_RETURN_MEAN
    from ray_amd.rllib.utils.pre_checks import check_env
    from ray_amd.rllib.utils.schedules import LinearSchedule, PiecewiseSchedule

    s = PiecewiseSchedule([(0, 1.0), (100, 0.1)], outside_value=0.1)
    assert s(0) == 1.0 and abs(s(50) - 0.55) < 1e-9 and s(1000) == 0.1
    assert LinearSchedule(10, 0.0)(5) == 0.5
    assert (ENV_RUNNER_RESULTS, EPISODE_RETURN_MEAN) == ("env_runners", "episode_return_mean")
    check_env(make_env("CartPole-v1", {}))
    np.testing.assert_allclose(discount_cumsum(np.ones(3), 0.5), [1.75, 1.5, 1.0])
    b = compute_advantages({"rewards": np.array([1.0, 1.0]), "vf_preds": np.array([0.5, 0.5])},
                           last_r=0.0, gamma=1.0, lambda_=1.0)
    np.testing.assert_allclose(b[Postprocessing.VALUE_TARGETS], [2.0, 1.0])
    np.testing.assert_allclose(b[Postprocessing.ADVANTAGES], [1.5, 0.5])


def test_alias_packages_and_atari_wrappers():
    from ray_amd.rllib.algorithms.appo import APPOConfig  # noqa: F401
    from ray_amd.rllib.algorithms.bc import BCConfig  # noqa: F401
    from ray_amd.rllib.env import spaces
    from ray_amd.rllib.env.envs import Env
    from ray_amd.rllib.env.wrappers.atari_wrappers import wrap_deepmind

    class Raw(Env):
        def __init__(self):
            self.observation_space = spaces.Box(0, 255, (210, 160, 3), np.uint8)
            self.action_space = spaces.Discrete(4)
            self.t = 0

        def reset(self, *, seed=None, options=None):
            self.t = 0
            return np.full((210, 160, 3), 128, np.uint8), {}

        def step(self, a):
            self.t += 1
            return np.full((210, 160, 3), 128, np.uint8), 5.0, self.t > 40, False, {}

    e = wrap_deepmind(Raw())
    o, _ = e.reset(seed=0)
    assert o.shape == (84, 84, 4) and o.dtype == np.uint8 and int(o[0, 0, 0]) == 128
    _, r, _, _, _ = e.step(0)
    assert r == 1.0  # clipped
