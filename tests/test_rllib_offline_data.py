"""Offline RL on ray_amd.data and off-policy estimation (modelled on rllib/offline/tests/
test_offline_data.py, rllib/algorithms/bc/tests, marwil/tests and rllib/offline/
estimators/tests/test_ope.py): transition Parquet written by EnvRunners, BC / MARWIL
trained from a Parquet directory (one local learner and two gloo learners over
streaming_split shards), IS / WIS checked against a numpy hand computation on a logged
CartPole dataset, DM / DR through FQE, and OPE wired to evaluation()."""

import glob
import os

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.rllib.algorithms import BCConfig, MARWILConfig, PPOConfig
from ray_amd.rllib.env import make_env
from ray_amd.rllib.offline import (DirectMethod, DoublyRobust, ImportanceSampling, JsonWriter,
                                   OfflineData, ParquetWriter, WeightedImportanceSampling,
                                   read_offline_dataset)


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6)
    yield
    ray.shutdown()


def _behaviour(o, rng):
    """A stochastic CartPole behaviour policy with known action probabilities."""
    p1 = 1.0 / (1.0 + np.exp(-4.0 * (o[2] + 0.5 * o[3])))
    a = int(rng.random() < p1)
    return a, (p1 if a == 1 else 1.0 - p1)


def _target_probs(obs):
    """Target policy for OPE: pi(a=1 | s) = sigmoid(6 (theta + 0.5 theta_dot))."""
    obs = np.asarray(obs)
    p1 = 1.0 / (1.0 + np.exp(-6.0 * (obs[:, 2] + 0.5 * obs[:, 3])))
    return np.stack([1.0 - p1, p1], 1)


def _log(path, writer_cls, n_frag=6, T=100, B=3, seed=0):
    """Record [T, B] fragments (with action_logp) through the given writer; returns the
    raw fragments for hand computations."""
    envs = [make_env("CartPole-v1") for _ in range(B)]
    obs = [e.reset(seed=seed + i)[0] for i, e in enumerate(envs)]
    w = writer_cls(str(path))
    rng = np.random.default_rng(seed)
    frags = []
    for _ in range(n_frag):
        cols = {k: np.zeros((T, B) + s, dt) for k, s, dt in (
            ("obs", (4,), np.float32), ("next_obs", (4,), np.float32),
            ("actions", (), np.int64), ("rewards", (), np.float32),
            ("terminateds", (), np.float32), ("truncateds", (), np.float32),
            ("action_logp", (), np.float32))}
        for t in range(T):
            for i, e in enumerate(envs):
                a, p = _behaviour(obs[i], rng)
                o2, r, te, tr, _ = e.step(a)
                cols["obs"][t, i], cols["actions"][t, i], cols["rewards"][t, i] = obs[i], a, r
                cols["terminateds"][t, i], cols["truncateds"][t, i] = float(te), float(tr)
                cols["next_obs"][t, i] = o2
                cols["action_logp"][t, i] = np.log(p)
                obs[i] = e.reset()[0] if (te or tr) else o2
        w.write(cols)
        frags.append(cols)
    if hasattr(w, "flush"):
        w.flush()
    return frags


def _episodes_by_hand(frags):
    """Complete episodes of the fragments: per env column, split at done."""
    B = frags[0]["rewards"].shape[1]
    eps = []
    for i in range(B):
        cur = {"obs": [], "actions": [], "rewards": [], "p": []}
        for f in frags:
            for t in range(f["rewards"].shape[0]):
                cur["obs"].append(f["obs"][t, i])
                cur["actions"].append(f["actions"][t, i])
                cur["rewards"].append(f["rewards"][t, i])
                cur["p"].append(np.exp(f["action_logp"][t, i]))
                if f["terminateds"][t, i] or f["truncateds"][t, i]:
                    eps.append({k: np.asarray(v) for k, v in cur.items()})
                    cur = {k: [] for k in cur}
        if cur["rewards"]:
            eps.append({k: np.asarray(v) for k, v in cur.items()})
    return eps


def test_parquet_transitions_roundtrip_with_episode_ids(cluster, tmp_path):
    frags = _log(tmp_path, ParquetWriter, n_frag=2, T=50, B=2)
    files = glob.glob(os.path.join(tmp_path, "*.parquet"))
    assert files
    ds = read_offline_dataset(str(tmp_path))
    rows = ds.take_all()
    assert len(rows) == 200 and rows[0]["obs"].shape == (4,)
    assert {"eps_id", "t", "action_prob", "next_obs"} <= set(rows[0])
    # episode ids and steps follow the env streams across the fragment boundary
    n_eps = len(_episodes_by_hand(frags))
    assert len({r["eps_id"] for r in rows}) == n_eps
    # the JSON fragment form reads into the same rows
    _log(tmp_path / "js", JsonWriter, n_frag=2, T=50, B=2)
    js = read_offline_dataset(str(tmp_path / "js")).take_all()
    assert len(js) == 200 and set(rows[0]) == set(js[0])
    d = OfflineData(str(tmp_path), gamma=0.9, seed=0)
    assert len(d) == 200
    b = d.sample(32)
    assert b["obs"].shape == (32, 4) and b["returns"].shape == (32,)
    # returns-to-go within an episode: R_t = r_t + 0.9 R_{t+1}; CartPole pays 1 per step
    assert np.all(b["returns"] >= 1.0 - 1e-6) and np.all(b["returns"] <= 10.0 + 1e-4)


def test_is_and_wis_match_a_numpy_hand_computation(cluster, tmp_path):
    frags = _log(tmp_path, JsonWriter, n_frag=4, T=80, B=3, seed=1)
    eps = _episodes_by_hand(frags)
    gamma = 0.95
    rows = {}
    for b in read_offline_dataset(str(tmp_path)).iter_batches(batch_size=100000):
        for k, v in b.items():
            rows.setdefault(k, []).append(v)
    batch = {k: np.concatenate(v) for k, v in rows.items()}
    # by hand
    vb, v_is, ps = [], [], []
    for e in eps:
        new = _target_probs(e["obs"])[np.arange(len(e["actions"])), e["actions"]]
        p = np.cumprod(new / e["p"])
        disc = gamma ** np.arange(len(p))
        vb.append((disc * e["rewards"]).sum())
        v_is.append((disc * p * e["rewards"]).sum())
        ps.append(p)
    L = max(len(p) for p in ps)
    wsum, wcnt = np.zeros(L), np.zeros(L)
    for p in ps:
        wsum[:len(p)] += p
        wcnt[:len(p)] += 1
    w = wsum / wcnt
    v_wis = [(gamma ** np.arange(len(p)) * p / w[:len(p)] * e["rewards"]).sum()
             for p, e in zip(ps, eps)]
    is_est = ImportanceSampling(_target_probs, gamma=gamma).estimate(batch)
    wis_est = WeightedImportanceSampling(_target_probs, gamma=gamma).estimate(batch)
    np.testing.assert_allclose(is_est["v_behavior"], np.mean(vb), rtol=1e-6)
    np.testing.assert_allclose(is_est["v_target"], np.mean(v_is), rtol=1e-6)
    np.testing.assert_allclose(is_est["v_target_std"], np.std(v_is), rtol=1e-6)
    np.testing.assert_allclose(wis_est["v_target"], np.mean(v_wis), rtol=1e-6)
    np.testing.assert_allclose(is_est["v_gain"], np.mean(v_is) / np.mean(vb), rtol=1e-6)
    # the target policy equal to the behaviour policy: IS is exact (ratios 1)
    same = ImportanceSampling(lambda o: np.stack(
        [1 - 1 / (1 + np.exp(-4 * (o[:, 2] + 0.5 * o[:, 3]))),
         1 / (1 + np.exp(-4 * (o[:, 2] + 0.5 * o[:, 3])))], 1), gamma=gamma).estimate(batch)
    np.testing.assert_allclose(same["v_target"], same["v_behavior"], rtol=1e-4)


def test_dm_and_dr_fit_fqe(cluster, tmp_path):
    _log(tmp_path, JsonWriter, n_frag=3, T=60, B=2, seed=2)
    ds = read_offline_dataset(str(tmp_path))

    class P:  # target policy object with an action space (FQE needs the action count)
        action_space = make_env("CartPole-v1").action_space

        def compute_log_likelihoods(self, actions, obs):
            return np.log(_target_probs(obs)[np.arange(len(actions)),
                                             np.asarray(actions).astype(int)])

    cfg = {"n_iters": 30, "lr": 3e-3, "minibatch_size": 64}
    dm = DirectMethod(P(), gamma=0.9, q_model_config=dict(cfg))
    dr = DoublyRobust(P(), gamma=0.9, q_model_config=dict(cfg))
    est_dm = dm.estimate_on_dataset(ds)
    est_dr = dr.estimate_on_dataset(ds)
    for e in (est_dm, est_dr):
        assert np.isfinite(e["v_target"]) and np.isfinite(e["v_behavior"])
    # CartPole pays 1 per step: V^pi of gamma 0.9 lies in (0, 10]
    assert 0.0 < est_dm["v_target"] <= 10.5 and 0.0 < est_dr["v_target"] <= 10.5
    losses = dm.model.train({k: v for k, v in next(ds.iter_batches(batch_size=10000)).items()})
    assert losses and np.all(np.isfinite(losses))


@pytest.mark.parametrize("learners", [0, 2])
def test_bc_and_marwil_train_from_parquet_through_ray_data(cluster, tmp_path, learners):
    _log(tmp_path, ParquetWriter, n_frag=4, T=100, B=2, seed=3)
    for cfg in (BCConfig(), MARWILConfig()):
        cfg = (cfg.environment("CartPole-v1")
               .offline_data(input_=str(tmp_path), input_read_method="read_parquet")
               .learners(num_learners=learners, num_gpus_per_learner=0)
               .training(train_batch_size=64, lr=1e-3, model={"fcnet_hiddens": [32]},
                         learner_backend="gloo")
               .debugging(seed=0))
        # two learners: 400-row shards = 12 batches of 32 per epoch, so 2 x 20 updates
        # run through several epochs of the streaming_split shards
        cfg.updates_per_iteration = 5 if not learners else 20
        cfg.eval_steps_per_iteration = 0
        algo = cfg.build()
        try:
            w0 = {k: np.array(v, copy=True) for k, v in algo.get_weights().items()}
            res = algo.train()
            if learners:
                res = algo.train()
            loss = res["learners"].get("policy_loss", res["learners"].get("total_loss"))
            assert np.isfinite(loss)
            w1 = algo.get_weights()
            assert any(not np.array_equal(w0[k], np.asarray(w1[k])) for k in w0)
            if learners:
                ws = algo.learner_group.foreach_learner(
                    lambda lr: {k: v.detach().numpy().copy()
                                for k, v in lr.module.state_dict().items()})
                for k in ws[0]:
                    np.testing.assert_array_equal(ws[0][k], ws[1][k])
        finally:
            algo.stop()


def test_ope_through_evaluation_config(cluster, tmp_path):
    _log(tmp_path / "train", ParquetWriter, n_frag=2, T=100, B=2, seed=4)
    _log(tmp_path / "eval", JsonWriter, n_frag=2, T=80, B=2, seed=5)
    cfg = (BCConfig().environment("CartPole-v1")
           .offline_data(input_=str(tmp_path / "train"))
           .learners(num_gpus_per_learner=0)
           .training(train_batch_size=64, model={"fcnet_hiddens": [16]})
           .evaluation(evaluation_interval=1,
                       evaluation_config={"input_": str(tmp_path / "eval")},
                       off_policy_estimation_methods={
                           "is": {"type": ImportanceSampling},
                           "wis": {"type": "WeightedImportanceSampling"},
                           "dm": {"type": DirectMethod, "q_model_config": {"n_iters": 5}},
                           "dr": {"type": "dr", "q_model_config": {"n_iters": 5}}})
           .debugging(seed=0))
    cfg.eval_steps_per_iteration = 0
    cfg.updates_per_iteration = 2
    algo = cfg.build()
    try:
        res = algo.train()
        ope = res["evaluation"]["off_policy_estimator"]
        assert set(ope) == {"is", "wis", "dm", "dr"}
        for v in ope.values():
            assert {"v_behavior", "v_target", "v_gain", "v_delta"} <= set(v)
            assert np.isfinite(v["v_target"])
        # the behaviour value is the logged data's, identical for every estimator
        assert len({round(v["v_behavior"], 6) for v in ope.values()}) == 1
    finally:
        algo.stop()


def test_env_runner_writes_parquet(cluster, tmp_path):
    cfg = (PPOConfig().environment("CartPole-v1").env_runners(num_env_runners=0)
           .offline_data(output=str(tmp_path), output_write_method="write_parquet",
                         output_max_rows_per_file=150)
           .learners(num_gpus_per_learner=0)
           .training(train_batch_size=200, minibatch_size=64, num_epochs=1,
                     model={"fcnet_hiddens": [16]}))
    algo = cfg.build()
    try:
        algo.train()
    finally:
        algo.stop()
    rows = read_offline_dataset(str(tmp_path)).take_all()
    assert len(rows) >= 150 and "action_prob" in rows[0]
    assert all(0.0 < r["action_prob"] <= 1.0 for r in rows)
