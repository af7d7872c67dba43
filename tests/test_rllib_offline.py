"""Off-policy / offline RLlib tests on CPU (modelled on rllib/algorithms/sac/tests/
test_sac.py, bc/tests/test_bc.py, marwil/tests/test_marwil.py, cql/tests/test_cql.py
and rllib/offline/tests): SAC steps on Pendulum, BC imitates a scripted CartPole
expert recorded through JsonWriter, MARWIL and CQL train from recorded data,
EnvRunners record through config.offline_data(output=...)."""

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.rllib.algorithms import BCConfig, CQLConfig, MARWILConfig, PPOConfig, SACConfig
from ray_amd.rllib.env import make_env
from ray_amd.rllib.offline import JsonReader, JsonWriter, OfflineData


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def _record(env_name, policy, path, n_frag=12, T=200, B=2, seed=0):
    envs = [make_env(env_name) for _ in range(B)]
    obs = [e.reset(seed=seed + i)[0] for i, e in enumerate(envs)]
    w = JsonWriter(str(path))
    rng = np.random.default_rng(seed)
    for _ in range(n_frag):
        cols = {k: [] for k in ("obs", "actions", "rewards", "terminateds", "truncateds",
                                "next_obs")}
        for _t in range(T):
            acts = [policy(o, rng) for o in obs]
            row = {k: [] for k in cols}
            for i, e in enumerate(envs):
                o2, r, te, tr, _ = e.step(acts[i])
                row["obs"].append(obs[i]), row["actions"].append(acts[i])
                row["rewards"].append(r), row["terminateds"].append(float(te))
                row["truncateds"].append(float(tr)), row["next_obs"].append(o2)
                obs[i] = e.reset()[0] if (te or tr) else o2
            for k in cols:
                cols[k].append(np.asarray(row[k]))
        w.write({k: np.stack(v).astype(np.float32 if k != "actions" or
                                       np.asarray(v).dtype.kind == "f" else np.int64)
                 for k, v in cols.items()})


def _cartpole_expert(o, rng):
    return int(o[2] + 0.5 * o[3] > 0)


def test_json_roundtrip(cluster, tmp_path):
    _record("CartPole-v1", _cartpole_expert, tmp_path, n_frag=2, T=50)
    bs = list(JsonReader(str(tmp_path)))
    assert len(bs) == 2 and bs[0]["obs"].shape == (50, 2, 4) and bs[0]["actions"].dtype == np.int64
    d = OfflineData(str(tmp_path), gamma=0.9)
    assert len(d) == 200 and d.sample(16)["returns"].shape == (16,)


def test_bc_imitates_scripted_expert(cluster, tmp_path):
    _record("CartPole-v1", _cartpole_expert, tmp_path)
    cfg = (BCConfig().environment("CartPole-v1").offline_data(input_=str(tmp_path))
           .training(lr=3e-3, train_batch_size=512, updates_per_iteration=50,
                     model={"fcnet_hiddens": [64, 64]})
           .env_runners(num_env_runners=0).debugging(seed=0))
    cfg.eval_steps_per_iteration = 1000
    algo = cfg.build()
    best = 0
    for _ in range(15):
        r = algo.train()
        m = r["env_runners"]["episode_return_mean"]
        if not np.isnan(m):
            best = max(best, m)
        if best > 300:
            break
    assert best > 250, best
    algo.stop()


def test_marwil_trains(cluster, tmp_path):
    _record("CartPole-v1", lambda o, rng: _cartpole_expert(o, rng) if rng.random() < 0.8
            else int(rng.integers(2)), tmp_path, n_frag=4)
    cfg = (MARWILConfig().environment("CartPole-v1").offline_data(input_=str(tmp_path))
           .training(lr=1e-3, beta=1.0, train_batch_size=256).env_runners(num_env_runners=0))
    algo = cfg.build()
    for _ in range(3):
        r = algo.train()
    assert np.isfinite(r["learners"]["total_loss"]) and "vf_loss" in r["learners"]
    algo.stop()


def test_sac_pendulum_runs(cluster):
    cfg = (SACConfig().environment("Pendulum-v1")
           .env_runners(num_env_runners=1, rollout_fragment_length=100)
           .training(num_steps_sampled_before_learning_starts=200, train_batch_size=64)
           .debugging(seed=0))
    algo = cfg.build()
    for _ in range(3):
        r = algo.train()
    lr = r["learners"]
    assert np.isfinite(lr["critic_loss"]) and 0 < lr["alpha_value"] < 1.0
    a = algo.compute_single_action(np.array([1.0, 0.0, 0.0], np.float32))
    assert a.shape == (1,) and -2.0 <= a[0] <= 2.0
    ck = algo.save()
    algo.restore(ck)
    algo.stop()


def test_cql_from_recorded_sac_rollouts(cluster, tmp_path):
    # record through EnvRunners: config.offline_data(output=...)
    cfg = (SACConfig().environment("Pendulum-v1").offline_data(output=str(tmp_path))
           .env_runners(num_env_runners=0, rollout_fragment_length=200)
           .training(num_steps_sampled_before_learning_starts=10_000))
    algo = cfg.build()
    for _ in range(3):
        algo.train()
    algo.stop()
    assert len(OfflineData(str(tmp_path))) == 600
    cq = (CQLConfig().environment("Pendulum-v1").offline_data(input_=str(tmp_path))
          .training(train_batch_size=64, bc_iters=5, updates_per_iteration=10)
          .env_runners(num_env_runners=0))
    algo = cq.build()
    for _ in range(2):
        r = algo.train()
    assert np.isfinite(r["learners"]["critic_loss"]) and np.isfinite(r["learners"]["actor_loss"])
    algo.stop()


PPOConfig  # noqa: B018
