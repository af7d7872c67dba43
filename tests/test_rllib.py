"""RLlib tests on CPU (modelled on rllib/algorithms/ppo/tests/test_ppo.py,
impala/tests, dqn/tests, utils/replay_buffers/tests)."""

import numpy as np
import pytest
import torch

import ray_amd as ray
from ray_amd.ops import reference as ref
from ray_amd.rllib.algorithms import APPOConfig, DQNConfig, IMPALAConfig, PPOConfig
from ray_amd.rllib.env import make_env
from ray_amd.rllib.utils.replay_buffers import (PrioritizedReplayBuffer, ReplayBuffer,
                                                ReservoirReplayBuffer, SumSegmentTree)


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6)
    yield
    ray.shutdown()


def test_envs():
    e = make_env("CartPole-v1")
    o, _ = e.reset(seed=0)
    assert o.shape == (4,)
    tot = 0
    for _ in range(600):
        o, r, te, tr, _ = e.step(e.action_space.sample())
        tot += r
        if te or tr:
            break
    assert 5 <= tot <= 500
    a = make_env("SyntheticAtari-v0")
    o, _ = a.reset()
    assert o.shape == (84, 84, 4) and o.dtype == np.uint8 and a.action_space.n == 6


def test_gae_reference_matches_rllib_formula():
    # single trajectory, compare with the discounted-cumsum formulation of
    # rllib/evaluation/postprocessing.py:compute_advantages
    T = 20
    rng = np.random.default_rng(0)
    r = rng.standard_normal(T)
    v = rng.standard_normal(T)
    last = 0.7
    gamma, lam = 0.99, 0.95
    vp = np.concatenate([v, [last]])
    delta = r + gamma * vp[1:] - vp[:-1]
    adv = np.zeros(T)
    acc = 0.0
    for t in range(T - 1, -1, -1):
        acc = delta[t] + gamma * lam * acc
        adv[t] = acc
    a, vt = ref.gae(torch.tensor(r)[:, None], torch.tensor(v)[:, None], torch.zeros(T, 1),
                    torch.tensor([last], dtype=torch.float64), gamma, lam)
    assert np.allclose(a[:, 0].numpy(), adv, atol=1e-5)
    assert np.allclose(vt[:, 0].numpy(), adv + v, atol=1e-5)


def test_ppo_cartpole_learns(cluster):
    cfg = (PPOConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=2, num_envs_per_env_runner=4)
           .training(train_batch_size=4000, minibatch_size=256, num_epochs=10, lr=3e-4,
                     gamma=0.99, lambda_=0.95, entropy_coeff=0.0, vf_loss_coeff=0.5,
                     clip_param=0.2, model={"fcnet_hiddens": [64, 64]})
           .debugging(seed=0))
    algo = cfg.build()
    first = None
    best = 0
    for i in range(12):
        r = algo.train()
        m = r["env_runners"]["episode_return_mean"]
        if first is None and not np.isnan(m):
            first = m
        best = max(best, m)
        if best > 150:
            break
    assert r["num_env_steps_sampled_lifetime"] >= 4000
    assert best > max(80, 2 * first), (first, best)
    ck = algo.save()
    w0 = algo.get_weights()
    algo.stop()
    algo2 = cfg.build()
    algo2.restore(ck)
    w1 = algo2.get_weights()
    assert all(torch.allclose(w0[k], w1[k]) for k in w0)
    a = algo2.compute_single_action(np.zeros(4, np.float32))
    assert a in (0, 1)
    algo2.stop()


def test_ppo_continuous_runs(cluster):
    cfg = (PPOConfig().environment("Pendulum-v1").env_runners(num_env_runners=1)
           .training(train_batch_size=400, minibatch_size=100, num_epochs=2))
    algo = cfg.build()
    r = algo.train()
    assert np.isfinite(r["learners"]["total_loss"])
    algo.stop()


@pytest.mark.parametrize("cfg_cls", [IMPALAConfig, APPOConfig])
def test_impala_appo_run(cluster, cfg_cls):
    cfg = (cfg_cls().environment("CartPole-v1")
           .env_runners(num_env_runners=2, num_envs_per_env_runner=2,
                        rollout_fragment_length=50)
           .training(train_batch_size=200, lr=5e-4))
    algo = cfg.build()
    for _ in range(3):
        r = algo.train()
    assert r["num_env_steps_sampled_lifetime"] >= 600
    assert np.isfinite(r["learners"]["total_loss"])
    algo.stop()


def test_dqn_runs(cluster):
    cfg = (DQNConfig().environment("CartPole-v1").env_runners(num_env_runners=0)
           .training(num_steps_sampled_before_learning_starts=100, train_batch_size=32))
    algo = cfg.build()
    for _ in range(60):
        r = algo.train()
    assert "loss" in r["learners"]
    algo.stop()


def test_replay_buffers():
    rb = ReplayBuffer(100, seed=0)
    rb.add({"x": np.arange(150), "y": np.arange(150) * 2})
    assert len(rb) == 100
    s = rb.sample(10)
    assert np.all(s["y"] == 2 * s["x"]) and s["x"].min() >= 50
    prb = PrioritizedReplayBuffer(64, alpha=1.0, seed=0)
    prb.add({"x": np.arange(64)})
    prb.update_priorities(np.arange(64), np.where(np.arange(64) == 7, 1000.0, 0.001))
    s = prb.sample(200)
    assert (s["x"] == 7).mean() > 0.9
    st = SumSegmentTree(8)
    st[np.arange(8)] = np.arange(8)
    assert st.sum() == 28
    assert st.find_prefixsum_idx([0.5])[0] == 1
    res = ReservoirReplayBuffer(10, seed=0)
    res.add({"x": np.arange(1000)})
    assert len(res) == 10


def _learner_weights(algo):
    from ray_amd.rllib.core.learner import _learner_call

    return [ray.get(a.execute.remote(_learner_call, "get_weights"))
            for a in algo.learner_group.actors]


def test_ppo_two_learners_gloo_uneven_shards(cluster):
    """num_learners=2 on gloo with 3 runners x 3 envs (9 columns -> 5/4 split): both ranks
    must run the same number of SGD steps (else the bucketed all-reduce deadlocks) and
    end with identical weights."""
    cfg = (PPOConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=3, num_envs_per_env_runner=3, rollout_fragment_length=37)
           .learners(num_learners=2, num_gpus_per_learner=0)
           .training(train_batch_size=333, minibatch_size=64, num_epochs=2,
                     model={"fcnet_hiddens": [32]}))
    algo = cfg.build()
    for _ in range(2):
        r = algo.train()
    assert np.isfinite(r["learners"]["total_loss"])
    w = _learner_weights(algo)
    assert all(torch.equal(w[0][k], w[1][k]) for k in w[0])
    algo.stop()


def test_impala_two_learners_gloo(cluster):
    cfg = (IMPALAConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=3, num_envs_per_env_runner=1, rollout_fragment_length=20)
           .learners(num_learners=2, num_gpus_per_learner=0)
           .training(train_batch_size=60, lr=5e-4))
    algo = cfg.build()
    for _ in range(2):
        r = algo.train()
    assert np.isfinite(r["learners"]["total_loss"])
    w = _learner_weights(algo)
    assert all(torch.equal(w[0][k], w[1][k]) for k in w[0])
    algo.stop()


def test_learner_state_roundtrip_is_lossless():
    """get_state carries the fp32 master, so save/restore continues bit-identically."""
    from ray_amd.rllib.core.learner import Learner

    env = make_env("CartPole-v1")
    cfg = {"model": {"fcnet_hiddens": [16]}, "lr": 1e-3, "num_gpus_per_learner": 0}
    a = Learner(cfg, env.observation_space, env.action_space, device=torch.device("cpu"))
    with torch.no_grad():
        a.flat.p32.add_(1e-9)  # sub-ulp master detail that a weights-only state would drop
    st = a.get_state()
    b = Learner(cfg, env.observation_space, env.action_space, device=torch.device("cpu"))
    b.set_state(st)
    assert torch.equal(a.flat.p32, b.flat.p32)


def test_ppo_sample_async_overlaps_and_counts_exactly(cluster):
    from ray_amd.rllib.algorithms import PPOConfig

    cfg = (PPOConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=2, num_envs_per_env_runner=2, sample_async=True)
           .learners(num_gpus_per_learner=0)
           .training(train_batch_size=200, minibatch_size=100, num_epochs=1,
                     model={"fcnet_hiddens": [16]}))
    algo = cfg.build()
    assert algo.config.rollout_fragment_length == 50  # auto: 200 / (2 runners x 2 envs)
    for _ in range(3):
        r = algo.train()
        assert r["num_env_steps_sampled_this_iter"] == 200
        assert "sample_wait_s" in r["learners"]
    assert r["env_runners"]["num_episodes"] > 0
    algo.stop()


def test_sample_actions_matches_categorical():
    """Gumbel-max sampling draws from softmax(logits); logp is the log-prob of the draw."""
    import torch

    from ray_amd.rllib.core.rl_module import RLModule
    from ray_amd.rllib.env import spaces

    m = RLModule(spaces.Box(-1, 1, (4,)), spaces.Discrete(4), {})
    torch.manual_seed(0)
    logits = torch.tensor([[2.0, 0.5, -1.0, 0.0]]).repeat(40000, 1)
    a, logp = m.sample_actions(logits, explore=True)
    freq = torch.bincount(a, minlength=4).float() / a.numel()
    p = torch.softmax(logits[0], -1)
    assert torch.allclose(freq, p, atol=0.01)
    assert torch.allclose(logp, torch.log(p)[a], atol=1e-6)
    a2, _ = m.sample_actions(logits[:3], explore=False)
    assert a2.tolist() == [0, 0, 0]


def test_fragments_staging_matches_concatenate():
    """Runner fragments assembled row-block-wise (native strided copy) == np.concatenate."""
    from ray_amd._native import _core
    from ray_amd.rllib.core.learner import Fragments, concat_batches

    rng = np.random.default_rng(0)
    parts = [rng.integers(0, 256, (7, b, 6, 6, 4), dtype=np.uint8) for b in (3, 5, 2)]
    batches = [{"obs": p, "rewards": np.ones((7, p.shape[1]), np.float32)} for p in parts]
    b = concat_batches(batches, lazy=("obs",))
    fr = b["obs"]
    assert isinstance(fr, Fragments) and fr.shape == (7, 10, 6, 6, 4)
    ref = np.concatenate(parts, axis=1)
    assert np.array_equal(np.asarray(fr), ref)
    dst = np.zeros(fr.shape, np.uint8)
    row = 6 * 6 * 4
    b0 = 0
    for p in fr.parts:
        _core.copy_rows(dst.reshape(-1), b0 * row, 10 * row, p.reshape(-1), p.shape[1] * row, 7,
                        p.shape[1] * row)
        b0 += p.shape[1]
    assert np.array_equal(dst, ref)
    with pytest.raises(IndexError):
        _core.copy_rows(dst.reshape(-1), 0, 10 * row, parts[0].reshape(-1), 3 * row, 8, 3 * row)
