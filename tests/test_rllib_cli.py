"""RLlib through Tune and the rllib CLI (modelled on rllib/tests/test_rllib_train_and_evaluate.py
and python/ray/tune/tests/test_api.py RLlib-trainable cases): string trainables with
old-stack config keys and nested stop criteria, class-trainable checkpoint frequency /
at-end, ``train``, ``train file`` and ``evaluate``."""

import json
import os
import subprocess
import sys
import tempfile

import pytest

import ray_amd as ray
from ray_amd import tune

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SMALL = {"num_workers": 1, "train_batch_size": 400, "sgd_minibatch_size": 64,
         "num_sgd_iter": 2}


@pytest.fixture()
def local_ray():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_tune_run_rllib_string_trainable_checkpoints(local_ray, tmp_path):
    ana = tune.run("PPO", config=dict(SMALL, env="CartPole-v1"),
                   stop={"timesteps_total": 1200, "sampler_results/episode_reward_mean": 1e9},
                   checkpoint_freq=2, checkpoint_at_end=True, storage_path=str(tmp_path),
                   name="ppo_str", verbose=0)
    (t,) = ana.trials
    assert t.error is None
    assert t.metrics["training_iteration"] == 3 and t.metrics["timesteps_total"] == 1200
    assert t.checkpoint is not None and t.checkpoint.path.endswith("checkpoint_000003")
    assert os.path.exists(os.path.join(t.checkpoint.path, "algorithm_state.pkl"))
    assert os.path.isdir(os.path.join(os.path.dirname(t.checkpoint.path),
                                      "checkpoint_000002"))  # checkpoint_freq=2


def test_tuner_with_algorithm_class_and_config_object(local_ray, tmp_path):
    from ray_amd.rllib.algorithms.ppo import PPO, PPOConfig
    from ray_amd.train import RunConfig

    cfg = (PPOConfig().environment("CartPole-v1").env_runners(num_env_runners=1)
           .training(train_batch_size=400, minibatch_size=64, num_epochs=1,
                     lr=tune.grid_search([1e-3, 1e-4])))
    grid = tune.Tuner(PPO, param_space=cfg, run_config=RunConfig(
        stop={"env_runners/num_episodes": 1}, storage_path=str(tmp_path))).fit()
    assert len(grid) == 2 and not grid.errors
    assert sorted(r.config["lr"] for r in grid) == [1e-4, 1e-3]


def _cli(*args, cwd=None, timeout=300):
    env = dict(os.environ, PYTHONPATH=REPO)
    env.pop("RAY_ADDRESS", None)
    return subprocess.run([sys.executable, "-m", "ray_amd.rllib", *args], env=env,
                          cwd=cwd, capture_output=True, text=True, timeout=timeout,
                          stdin=subprocess.DEVNULL)


def test_cli_train_file_then_evaluate():
    d = tempfile.mkdtemp(prefix="rllibcli")
    with open(os.path.join(d, "cartpole-ppo.yaml"), "w") as f:
        f.write("cartpole-ppo:\n"
                "    env: CartPole-v1\n"
                "    run: PPO\n"
                "    stop:\n"
                "        timesteps_total: 800\n"
                "    config:\n"
                "        framework: torch\n"
                "        gamma: 0.99\n"
                "        lr: 0.0003\n"
                "        num_workers: 1\n"
                "        num_sgd_iter: 2\n"
                "        sgd_minibatch_size: 64\n"
                "        train_batch_size: 400\n"
                "        model:\n"
                "            fcnet_hiddens: [32]\n")
    r = _cli("train", "file", "cartpole-ppo.yaml", "--checkpoint-at-end", "--storage-path",
             d, "--ray-num-cpus", "4", cwd=d)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["timesteps_total"] == 800 and line["checkpoint"]
    r = _cli("evaluate", line["checkpoint"], "--algo", "PPO", "--episodes", "3",
             "--ray-num-cpus", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    ev = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert ev["episodes"] == 3 and ev["env"] == "CartPole-v1"
    assert all(x >= 1 for x in ev["episode_returns"])


def test_cli_train_flags():
    d = tempfile.mkdtemp(prefix="rllibcli")
    r = _cli("train", "--algo", "PPO", "--env", "CartPole-v1", "--config",
             json.dumps(SMALL), "--stop", '{"training_iteration": 2}', "--storage-path", d,
             "--ray-num-cpus", "4", cwd=d)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["training_iteration"] == 2 and line["error"] is None
