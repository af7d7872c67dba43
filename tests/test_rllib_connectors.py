"""RLlib connectors, MeanStdFilter and callbacks (modelled on rllib/connectors/tests/,
rllib/utils/tests/test_filters.py and rllib/algorithms/tests/test_callbacks_on_*.py)."""

import numpy as np
import pytest
import torch

import ray_amd as ray
from ray_amd.rllib.algorithms import PPOConfig
from ray_amd.rllib.callbacks import RLlibCallback
from ray_amd.rllib.connectors import (ConnectorPipelineV2, ConnectorV2, FlattenObservations,
                                      MeanStdFilter, PrevActionsPrevRewards)


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


class AddOne(ConnectorV2):
    def __call__(self, *, batch, **kw):
        batch["obs"] = batch["obs"] + 1
        return batch


def test_pipeline_edit_operations():
    p = ConnectorPipelineV2(connectors=[AddOne(), FlattenObservations()])
    p.insert_after(AddOne, MeanStdFilter())
    p.insert_before("FlattenObservations", AddOne())
    assert [type(c).__name__ for c in p.connectors] == [
        "AddOne", "MeanStdFilter", "AddOne", "FlattenObservations"]
    p.remove("MeanStdFilter")
    out = p(batch={"obs": np.zeros((3, 2, 2), np.float32)})
    assert out["obs"].shape == (3, 4) and float(out["obs"].max()) == 2.0
    assert len(p.find(AddOne)) == 2


def test_ppo_learner_side_mean_std_filter(cluster):
    """The learner owns the statistics (HIP Welford kernel on GPU, same math on CPU), the
    runner normalizes with the broadcast copy."""
    cfg = (PPOConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=0, num_envs_per_env_runner=2,
                        observation_filter="MeanStdFilter")
           .learners(num_gpus_per_learner=0)
           .training(train_batch_size=256, minibatch_size=64, num_epochs=1,
                     model={"fcnet_hiddens": [16]}))
    algo = cfg.build()
    for _ in range(2):
        r = algo.train()
    lf = algo.learner_group.local.obs_filter
    assert lf is not None and lf.count >= 512
    rf_ = algo.local_runner._post[0].rms
    assert rf_.count == lf.count and torch.allclose(rf_.mean, lf.mean.cpu())
    # recorded observations stay raw; the module input is normalized
    b = algo.local_runner.sample(8)
    raw, norm = algo.local_runner._module_obs(b["bootstrap_obs"], False, update=False)
    assert np.allclose(raw, b["bootstrap_obs"]) and not np.allclose(norm, raw)
    assert np.isfinite(r["learners"]["total_loss"])
    a = algo.compute_single_action(np.zeros(4, np.float32))
    assert a in (0, 1)
    ck = algo.save()
    algo2 = cfg.build()
    algo2.restore(ck)
    assert algo2.learner_group.local.obs_filter.count == lf.count
    algo.stop()
    algo2.stop()


def test_env_to_module_connectors_change_module_input(cluster):
    cfg = (PPOConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=1, num_envs_per_env_runner=2,
                        env_to_module_connector=lambda env: [PrevActionsPrevRewards(
                            input_action_space=__import__(
                                "ray_amd.rllib.env.spaces", fromlist=["Discrete"]).Discrete(2))])
           .learners(num_gpus_per_learner=0)
           .training(train_batch_size=128, minibatch_size=64, num_epochs=1,
                     model={"fcnet_hiddens": [16]}))
    algo = cfg.build()
    assert algo.observation_space.shape == (4 + 2 + 1,)
    r = algo.train()
    assert np.isfinite(r["learners"]["total_loss"])
    algo.stop()


class CountingCallbacks(RLlibCallback):
    def __init__(self):
        self.inits = 0
        self.results = 0

    def on_algorithm_init(self, *, algorithm, **kw):
        self.inits += 1
        algorithm._cb_seen = self

    def on_episode_start(self, *, episode, **kw):
        episode.user_data["steps"] = 0

    def on_episode_step(self, *, episode, **kw):
        episode.user_data["steps"] += 1

    def on_episode_end(self, *, episode, metrics_logger=None, **kw):
        episode.custom_metrics["ep_steps_seen"] = episode.user_data["steps"]
        metrics_logger.log_value("episodes_done", 1, reduce="sum")

    def on_train_result(self, *, algorithm, result, **kw):
        self.results += 1
        result["callback_ok"] = True


def test_rllib_callbacks(cluster):
    cfg = (PPOConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=1, num_envs_per_env_runner=4)
           .learners(num_gpus_per_learner=0)
           .callbacks(CountingCallbacks)
           .training(train_batch_size=400, minibatch_size=100, num_epochs=1,
                     model={"fcnet_hiddens": [16]}))
    algo = cfg.build()
    r = algo.train()
    cb = algo._cb_seen
    assert cb.inits == 1 and cb.results == 1 and r["callback_ok"]
    cm = r["env_runners"]["custom_metrics"]
    assert cm["ep_steps_seen"] > 5 and cm["episodes_done"] >= 1
    algo.stop()
