"""DreamerV3 (modelled on rllib/algorithms/dreamerv3/tests/test_dreamerv3.py: build with a
tiny model, train a few iterations on discrete and continuous envs; plus world-model
and checkpoint sanity checks)."""

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.rllib.algorithms.dreamerv3 import DreamerV3Config


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=2)
    yield
    ray.shutdown()


def _cfg(env):
    return (DreamerV3Config().environment(env)
            .training(model_size="nano", batch_size_B=4, batch_length_T=16, horizon_H=5,
                      training_ratio=32, symlog_obs=True)
            .learners(num_gpus_per_learner=0).debugging(seed=0))


@pytest.mark.parametrize("env", ["CartPole-v1", "Pendulum-v1"])
def test_dreamerv3_compilation_and_training(cluster, env):
    algo = _cfg(env).build()
    for _ in range(3):
        r = algo.train()
    ls = r["learners"]
    assert r["num_env_steps_sampled_lifetime"] >= 64
    algo.train()
    keys = ("WORLD_MODEL_L_total", "CRITIC_L_total", "ACTOR_L_total")
    st = algo._update(algo.replay.sample(4, 16))
    for k in keys:
        assert np.isfinite(st[k]), (k, st)
    a = algo.compute_single_action(np.zeros(algo.observation_space.shape, np.float32))
    assert algo.action_space.contains(np.asarray(a, dtype=algo.action_space.dtype)
                                      if not isinstance(a, int) else a)
    ls  # noqa: B018
    algo.stop()


def test_world_model_fits_a_batch_and_checkpoints(cluster):
    import torch

    torch.manual_seed(0)  # the decrease over 40 steps at lr 1e-4 depends on the init
    algo = _cfg("CartPole-v1").build()
    algo.train()
    b = algo.replay.sample(4, 16)
    first = algo._update(b)["WORLD_MODEL_L_decoder"]
    for _ in range(80):
        last = algo._update(b)["WORLD_MODEL_L_decoder"]
    assert last < 0.8 * first, (first, last)  # lr 1e-4: a clear, not a full, decrease
    ck = algo.save()
    algo2 = _cfg("CartPole-v1").build()
    algo2.restore(ck)
    import torch

    for p1, p2 in zip(algo.world.parameters(), algo2.world.parameters()):
        assert torch.equal(p1, p2)
    assert algo2.replayed_steps == algo.replayed_steps
    algo.stop()
    algo2.stop()


@pytest.mark.gpu
def test_dreamerv3_on_gpu_learner(cluster):
    import torch

    algo = (_cfg("CartPole-v1").learners(num_gpus_per_learner=1)).build()
    assert algo.device.type == "cuda"
    algo.train()
    st = algo._update(algo.replay.sample(4, 16))
    assert np.isfinite(st["WORLD_MODEL_L_total"]) and np.isfinite(st["ACTOR_L_total"])
    assert next(algo.world.parameters()).is_cuda
    torch.cuda.synchronize()
    algo.stop()
