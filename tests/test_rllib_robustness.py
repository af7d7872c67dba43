"""RLlib robustness: EnvRunner fault tolerance (a killed runner is recreated with the
current weights), evaluation EnvRunners running in parallel with training, and the
N-learner IMPALA path where sample batches go straight to the learner actors (reference:
rllib/utils/actor_manager.py:193, algorithm_config.py:2673 fault_tolerance,
algorithm.py:642 evaluation workers, impala.py:130,194)."""
import pytest

import ray_amd as ray
from ray_amd.rllib.algorithms import IMPALAConfig, PPOConfig


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=8)
    yield
    ray.shutdown()


def _ppo(**ft):
    return (PPOConfig().environment("CartPole-v1")
            .env_runners(num_env_runners=2, num_envs_per_env_runner=2)
            .training(train_batch_size=400, minibatch_size=100, num_epochs=2)
            .fault_tolerance(**ft).debugging(seed=0))


def test_killed_env_runner_is_restored(cluster):
    algo = _ppo(restart_failed_env_runners=True).build()
    algo.train()
    victim = algo.env_runners[0]
    ray.kill(victim)
    for _ in range(3):
        r = algo.train()
    assert algo.num_env_runner_restarts >= 1
    assert r["num_healthy_env_runners"] == 2
    assert victim not in algo.env_runners
    # the replacement samples with the learner's weights (same version as the others)
    vs = ray.get([x.apply.remote(__import__("cloudpickle").dumps(
        lambda runner: runner.weights_version)) for x in algo.env_runners])
    assert len(set(vs)) == 1 and vs[0] == algo.weights_version
    algo.stop()


def test_ignore_env_runner_failures_keeps_training(cluster):
    algo = _ppo(restart_failed_env_runners=False, ignore_env_runner_failures=True).build()
    algo.train()
    ray.kill(algo.env_runners[1])
    r = None
    for _ in range(2):
        r = algo.train()
    assert r["num_healthy_env_runners"] == 1 and algo.num_env_runner_restarts == 0
    algo.stop()


def test_env_runner_failure_raises_without_tolerance(cluster):
    algo = _ppo(restart_failed_env_runners=False, ignore_env_runner_failures=False).build()
    algo.train()
    ray.kill(algo.env_runners[0])
    with pytest.raises(Exception):
        for _ in range(2):
            algo.train()
    algo.stop()


def test_parallel_evaluation_env_runners(cluster):
    cfg = (_ppo().evaluation(evaluation_interval=1, evaluation_duration=4,
                             evaluation_num_env_runners=2,
                             evaluation_parallel_to_training=True))
    algo = cfg.build()
    r = algo.train()
    ev = r["evaluation"]
    assert ev["num_evaluation_env_runners"] == 2
    assert ev["env_runners"]["num_episodes"] == 4
    assert ev["env_runners"]["episode_return_mean"] > 0
    # timesteps unit, sequential (no parallel flag) on the same evaluation runners
    algo.config.evaluation_duration_unit = "timesteps"
    algo.config.evaluation_duration = 300
    ev2 = algo.evaluate()
    assert ev2["env_runners"]["num_env_steps_sampled"] >= 300
    algo.stop()


def test_local_evaluation_runner_is_reused(cluster):
    algo = _ppo().evaluation(evaluation_interval=1, evaluation_duration=2).build()
    algo.train()
    first = algo._eval_local
    algo.train()
    assert first is not None and algo._eval_local is first
    algo.stop()


def test_impala_two_learners_batches_bypass_driver(cluster):
    cfg = (IMPALAConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=2, num_envs_per_env_runner=2,
                        rollout_fragment_length=25)
           .training(train_batch_size=200, learner_backend="gloo")
           .learners(num_learners=2, num_gpus_per_learner=0)
           .fault_tolerance(restart_failed_env_runners=True).debugging(seed=0))
    algo = cfg.build()
    stats = []
    for i in range(4):
        r = algo.train()
        stats.append(r["learners"])
        if i == 1:
            ray.kill(algo.env_runners[0])  # runner death mid-training: restored
    assert algo.num_driver_batch_fetches == 0
    assert any("total_loss" in s for s in stats)
    assert algo.num_env_runner_restarts >= 1
    assert r["num_env_steps_sampled_lifetime"] >= 800
    algo.stop()
