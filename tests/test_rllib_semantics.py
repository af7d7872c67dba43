"""RLlib algorithm lifecycle semantics (modelled on rllib/algorithms/tests/test_algorithm.py,
test_algorithm_save_load_checkpoint_learner.py, rllib/algorithms/ppo/tests/test_ppo.py,
rllib/utils/tests/test_filter*.py, rllib/evaluation tests): checkpoints round-trip,
deterministic inference, batch accounting, config plumbing."""

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.rllib.algorithms.dqn import DQNConfig
from ray_amd.rllib.algorithms.impala import IMPALAConfig
from ray_amd.rllib.algorithms.ppo import PPOConfig


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _ppo(**kw):
    return (PPOConfig().environment("CartPole-v1")
            .env_runners(num_env_runners=kw.pop("runners", 1), num_envs_per_env_runner=2)
            .training(train_batch_size=400, minibatch_size=100, num_epochs=2,
                      model={"fcnet_hiddens": [16]}, **kw)
            .debugging(seed=3))


def test_checkpoint_restore_continues_identically(cluster, tmp_path):
    algo = _ppo().build()
    algo.train()
    ck = algo.save(str(tmp_path / "ck"))
    w_saved = {k: np.array(v, np.float32) for k, v in algo.get_weights().items()
               if not k.startswith("__")}
    algo.stop()
    algo2 = _ppo().build()
    algo2.restore(ck)
    w2 = algo2.get_weights()
    assert all(np.array_equal(w_saved[k], np.asarray(w2[k], np.float32)) for k in w_saved)
    assert algo2.iteration == 1
    r = algo2.train()
    assert r["training_iteration"] == 2
    algo2.stop()


def test_from_checkpoint_rebuilds_config(cluster, tmp_path):
    from ray_amd.rllib.algorithms.ppo import PPO

    algo = _ppo(lr=1.234e-4).build()
    algo.train()
    ck = algo.save(str(tmp_path / "ck2"))
    algo.stop()
    algo2 = PPO.from_checkpoint(ck)
    assert np.isclose(algo2.config.lr, 1.234e-4)
    assert algo2.iteration == 1
    algo2.stop()


def test_greedy_action_is_deterministic(cluster):
    algo = _ppo().build()
    obs = np.array([0.01, -0.02, 0.03, 0.0], np.float32)
    acts = {algo.compute_single_action(obs, explore=False) for _ in range(10)}
    assert len(acts) == 1 and acts.pop() in (0, 1)
    algo.stop()


def test_ppo_iteration_samples_exactly_train_batch(cluster):
    algo = _ppo(runners=2).build()
    r = algo.train()
    assert r["num_env_steps_sampled_this_iter"] == 400
    r = algo.train()
    assert r["num_env_steps_sampled_lifetime"] == 800
    algo.stop()


def test_episode_metrics_and_smoothing_window(cluster):
    cfg = _ppo()
    cfg.metrics_num_episodes_for_smoothing = 5
    algo = cfg.build()
    for _ in range(3):
        r = algo.train()
    er = r["env_runners"]
    assert er["num_episodes"] <= 5 and er["episode_len_mean"] > 0
    assert er["episode_return_min"] <= er["episode_return_mean"] <= er["episode_return_max"]
    algo.stop()


def test_impala_learns_cartpole_quickly(cluster):
    cfg = (IMPALAConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=2, num_envs_per_env_runner=4, rollout_fragment_length=50)
           .training(train_batch_size=400, lr=1e-3, model={"fcnet_hiddens": [64]})
           .debugging(seed=0))
    algo = cfg.build()
    best = 0
    for _ in range(120):
        r = algo.train()
        m = r["env_runners"]["episode_return_mean"]
        if m == m:
            best = max(best, m)
        if best > 60:
            break
    algo.stop()
    assert best > 60, best


def test_dqn_epsilon_schedule_and_target_sync(cluster):
    cfg = (DQNConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=0, num_envs_per_env_runner=1)
           .training(train_batch_size=32, model={"fcnet_hiddens": [16]}))
    cfg.num_steps_sampled_before_learning_starts = 50
    cfg.epsilon = [(0, 1.0), (200, 0.1)]
    cfg.target_network_update_freq = 40
    algo = cfg.build()
    eps = []
    for _ in range(80):
        r = algo.train()
        eps.append(r["learners"]["epsilon"])
    assert eps[0] == pytest.approx(1.0, abs=0.05)
    assert eps[-1] == pytest.approx(0.1)
    assert all(a >= b - 1e-9 for a, b in zip(eps, eps[1:]))  # monotone decay
    assert "loss" in r["learners"]
    algo.stop()
