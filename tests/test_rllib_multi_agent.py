"""Multi-agent RLlib tests (modelled on rllib/env/tests/test_multi_agent_env.py and
rllib/examples/multi_agent/multi_agent_cartpole.py)."""

import numpy as np
import pytest

import ray_amd as ray
from ray_amd.rllib.algorithms.ppo import PPOConfig
from ray_amd.rllib.env import MultiAgentCartPole, make_multi_agent
from ray_amd.rllib.env.multi_agent_env_runner import MultiAgentEnvRunner


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


def test_make_multi_agent_env_semantics():
    env = MultiAgentCartPole({"num_agents": 3})
    obs, _ = env.reset(seed=1)
    assert set(obs) == {0, 1, 2} and env.get_agent_ids() == {0, 1, 2}
    done_all = False
    steps = 0
    while not done_all:
        o, r, te, tr, _ = env.step({a: 0 for a in env.agents})
        assert set(r) <= {0, 1, 2}
        done_all = te["__all__"]
        steps += 1
    assert 5 < steps < 500 and env.agents == []


def _runner_cfg(num_agents=3, mapping=None, policies=("p0", "p1")):
    env = MultiAgentCartPole({"num_agents": num_agents})
    specs = {p: (env.observation_space, env.action_space) for p in policies}
    return {"env": "MultiAgentCartPole", "env_config": {"num_agents": num_agents},
            "num_envs_per_env_runner": 2, "seed": 0, "_module_specs": specs,
            "policy_mapping_fn": mapping or (lambda aid, ep, **kw: f"p{aid % 2}"),
            "model": {"fcnet_hiddens": [16]}}


def test_runner_columns_padding_and_mask():
    r = MultiAgentEnvRunner(_runner_cfg(), 0)
    out = r.sample(120)
    assert out["env_steps"] == 240
    b0, b1 = out["modules"]["p0"], out["modules"]["p1"]
    # agents 0,2 -> p0 and agent 1 -> p1, in each of the 2 envs
    assert b0["obs"].shape[:2] == (120, 4) and b1["obs"].shape[:2] == (120, 2)
    for b in (b0, b1):
        m = b["loss_mask"]
        # every padding row is a terminal row (so GAE cannot cross it) with zero reward
        assert np.all(b["terminateds"][m == 0] == 1) and np.all(b["rewards"][m == 0] == 0)
        # CartPole: reward 1 on every acted step
        assert np.all(b["rewards"][m == 1] == 1)
    total_agent_steps = b0["loss_mask"].sum() + b1["loss_mask"].sum()
    assert total_agent_steps == out["agent_steps"] > 240
    # episodes ended, returns are summed over agents
    met = r.get_metrics()
    assert met["episode_returns"] and set(met["module_episode_returns"]) == {"p0", "p1"}


def test_runner_rejects_unknown_module():
    with pytest.raises(ValueError):
        MultiAgentEnvRunner(_runner_cfg(mapping=lambda aid, ep, **kw: "nope"), 0).sample(2)


def test_multi_agent_ppo_two_policies_learn(cluster, tmp_path):
    cfg = (PPOConfig().environment("MultiAgentCartPole", env_config={"num_agents": 2})
           .env_runners(num_env_runners=2, num_envs_per_env_runner=2)
           .multi_agent(policies={"p0", "p1"},
                        policy_mapping_fn=lambda aid, ep, **kw: f"p{aid}")
           .training(train_batch_size=2000, minibatch_size=256, num_epochs=8, lr=3e-4,
                     lambda_=0.95, vf_loss_coeff=0.5, clip_param=0.2,
                     model={"fcnet_hiddens": [64, 64]})
           .debugging(seed=0))
    algo = cfg.build()
    first, best = None, {}
    for _ in range(10):
        res = algo.train()
        mr = res["module_episode_returns_mean"]
        if first is None and len(mr) == 2:
            first = dict(mr)
        for k, v in mr.items():
            best[k] = max(best.get(k, 0), v)
        if best and min(best.values()) > 80:
            break
    assert {"p0", "p1"} <= set(res["learners"])
    assert all(best[k] > max(40, 1.5 * first[k]) for k in ("p0", "p1")), (first, best)
    w = algo.get_weights()
    assert set(w) == {"p0", "p1"}
    a = algo.compute_single_action(np.zeros(4, np.float32), policy_id="p1")
    assert a in (0, 1)
    ck = algo.save(str(tmp_path / "ck"))
    algo.stop()
    algo2 = cfg.build()
    algo2.restore(ck)
    w2 = algo2.get_weights()
    for mid in ("p0", "p1"):
        for k in w[mid]:
            assert np.allclose(np.asarray(w[mid][k], np.float32),
                               np.asarray(w2[mid][k], np.float32))
    algo2.stop()


def test_policies_to_train_freezes_others(cluster):
    cfg = (PPOConfig().environment("MultiAgentCartPole", env_config={"num_agents": 2})
           .env_runners(num_env_runners=0)
           .multi_agent(policies={"p0", "p1"}, policy_mapping_fn=lambda aid, ep, **kw: f"p{aid}",
                        policies_to_train=["p0"])
           .training(train_batch_size=400, minibatch_size=128, num_epochs=2,
                     model={"fcnet_hiddens": [16]}))
    algo = cfg.build()
    w0 = {m: {k: np.array(v, np.float32, copy=True) for k, v in w.items()}
          for m, w in algo.get_weights().items()}
    res = algo.train()
    w1 = algo.get_weights()
    assert "p0" in res["learners"] and "p1" not in res["learners"]
    k = next(iter(w0["p1"]))
    assert np.allclose(np.asarray(w0["p1"][k]), np.asarray(w1["p1"][k]))
    assert not all(np.allclose(np.asarray(w0["p0"][k2]), np.asarray(w1["p0"][k2]))
                   for k2 in w0["p0"])
    algo.stop()


def test_unsupported_multi_agent_rejected(cluster):
    from ray_amd.rllib.algorithms.marwil import MARWILConfig
    cfg = (MARWILConfig().environment("MultiAgentCartPole")
           .multi_agent(policies={"p0"}, policy_mapping_fn=lambda aid, ep, **kw: "p0"))
    with pytest.raises(NotImplementedError):
        cfg.build()


def test_multi_agent_sac_trains_each_module(cluster):
    """Continuous multi-agent SAC: per-module replay buffers and learners; the module left
    out of policies_to_train keeps its weights."""
    from ray_amd.rllib.algorithms.sac import SACConfig

    cfg = (SACConfig().environment("MultiAgentPendulum", env_config={"num_agents": 3})
           .env_runners(num_env_runners=0, num_envs_per_env_runner=2)
           .multi_agent(policies={"p0", "p1", "p2"},
                        policy_mapping_fn=lambda aid, ep, **kw: f"p{aid}",
                        policies_to_train=["p0", "p1"])
           .training(train_batch_size=32, model={"fcnet_hiddens": [32]})
           .debugging(seed=0))
    cfg.num_steps_sampled_before_learning_starts = 64
    cfg.rollout_fragment_length = 16
    algo = cfg.build()
    w0 = {m: {k: np.array(v, np.float32) for k, v in w.items()}
          for m, w in algo.get_weights().items()}
    for _ in range(6):
        res = algo.train()
    w1 = algo.get_weights()
    assert {"p0/critic_loss", "p1/critic_loss"} <= set(res["learners"])
    assert not any(k.startswith("p2/") for k in res["learners"])
    k = next(iter(w0["p2"]))
    assert np.allclose(w0["p2"][k], np.asarray(w1["p2"][k], np.float32))
    assert not all(np.allclose(w0["p0"][k2], np.asarray(w1["p0"][k2], np.float32))
                   for k2 in w0["p0"])
    assert res["env_runners"]["num_episodes"] >= 0
    algo.stop()


def test_make_multi_agent_from_creator():
    from ray_amd.rllib.env import CartPoleEnv
    cls = make_multi_agent(lambda cfg: CartPoleEnv(cfg))
    env = cls({"num_agents": 2})
    obs, _ = env.reset()
    assert set(obs) == {0, 1}


# ------------------------------------------------------------------ turn-based envs
def _guess_cfg(T_envs=2, length=10):
    from ray_amd.rllib.env import TurnBasedGuess

    env = TurnBasedGuess({"num_cues": 4, "episode_len": length})
    specs = {p: (env.observation_space, env.action_space) for p in ("p1", "p2")}
    return {"env": "TurnBasedGuess", "env_config": {"num_cues": 4, "episode_len": length},
            "num_envs_per_env_runner": T_envs, "seed": 3, "_module_specs": specs,
            "policy_mapping_fn": lambda aid, ep, **kw: aid, "model": {"fcnet_hiddens": [16]}}


def test_turn_based_runner_credits_delayed_rewards():
    """Rewards are paid one move late (after the opponent answers); every completed row
    must carry exactly the reward of ITS action, padding rows lead the column."""
    r = MultiAgentEnvRunner(_guess_cfg(), 0)
    acted = 0
    for frag in range(3):
        out = r.sample(25)
        for mid in ("p1", "p2"):
            b = out["modules"][mid]
            m = b["loss_mask"]
            assert b["obs"].shape[:2] == (25, 2)
            real = m == 1
            want = (b["obs"].argmax(-1) == b["actions"]).astype(np.float32)
            assert np.array_equal(b["rewards"][real], want[real])
            assert np.all(b["terminateds"][~real] == 1) and np.all(b["rewards"][~real] == 0)
            for j in range(m.shape[1]):  # right-aligned: no padding after a real row
                col = m[:, j]
                first = int(np.argmax(col)) if col.any() else len(col)
                assert np.all(col[first:] == 1)
            acted += int(m.sum())
    # 2 envs x 75 env steps = 150 moves; only the moves still pending are missing
    assert 146 <= acted <= 150
    # episodes of 10 moves: every player's 5 moves end in one terminal row
    b = out["modules"]["p1"]
    assert b["terminateds"][b["loss_mask"] == 1].sum() >= 1


def test_tictactoe_rules():
    from ray_amd.rllib.env import TicTacToe

    e = TicTacToe()
    o, _ = e.reset()
    assert set(o) == {"player1"}
    for cell, who in ((0, "player1"), (3, "player2"), (1, "player1"), (4, "player2")):
        o, r, te, _, _ = e.step({who: cell})
        assert not te["__all__"]
    o, r, te, _, _ = e.step({"player1": 2})  # top row
    assert te["__all__"] and r == {"player1": 1.0, "player2": -1.0}
    e.reset()
    e.step({"player1": 4})
    o, r, te, _, _ = e.step({"player2": 4})  # occupied
    assert te["__all__"] and r["player2"] == -1.0


def test_turn_based_ppo_learns(cluster):
    cfg = (PPOConfig().environment("TurnBasedGuess", env_config={"num_cues": 4,
                                                                "episode_len": 10})
           .env_runners(num_env_runners=0, num_envs_per_env_runner=4)
           .multi_agent(policies={"p1", "p2"}, policy_mapping_fn=lambda aid, ep, **kw: aid)
           .training(train_batch_size=800, minibatch_size=128, num_epochs=6, lr=3e-3,
                     gamma=0.9, lambda_=0.9, model={"fcnet_hiddens": [32]})
           .debugging(seed=0))
    algo = cfg.build()
    best = {}
    for _ in range(12):
        mr = algo.train()["module_episode_returns_mean"]
        for k, v in mr.items():
            best[k] = max(best.get(k, 0.0), v)
        if best and min(best.values()) > 4.0:
            break
    algo.stop()
    # random play earns 5 moves x 1/4; the optimum is 5 per player
    assert min(best.get("p1", 0), best.get("p2", 0)) > 3.5, best


def test_multi_agent_impala_learns(cluster):
    from ray_amd.rllib.algorithms.impala import IMPALAConfig

    cfg = (IMPALAConfig().environment("TurnBasedGuess", env_config={"num_cues": 4,
                                                                    "episode_len": 10})
           .env_runners(num_env_runners=1, num_envs_per_env_runner=4)
           .multi_agent(policies={"p1", "p2"}, policy_mapping_fn=lambda aid, ep, **kw: aid)
           .training(train_batch_size=400, lr=3e-3, gamma=0.9, entropy_coeff=0.0,
                     model={"fcnet_hiddens": [32]})
           .debugging(seed=0))
    cfg.rollout_fragment_length = 50
    algo = cfg.build()
    best = {}
    for _ in range(300):  # one V-trace SGD step per iteration
        res = algo.train()
        for k, v in res.get("module_episode_returns_mean", {}).items():
            best[k] = max(best.get(k, 0.0), v)
        if best and min(best.values()) > 4.0:
            break
    assert {"p1", "p2"} <= set(res["learners"])
    algo.stop()
    assert min(best.get("p1", 0), best.get("p2", 0)) > 3.5, best


def test_multi_agent_dqn_learns_turn_based(cluster):
    """Per-module replay buffers fed with completed agent rows (next_obs = the state the
    agent acts on next, across the opponent's move)."""
    from ray_amd.rllib.algorithms.dqn import DQNConfig

    cfg = (DQNConfig().environment("TurnBasedGuess", env_config={"num_cues": 4,
                                                                 "episode_len": 10})
           .env_runners(num_env_runners=0, num_envs_per_env_runner=4)
           .multi_agent(policies={"p1", "p2"}, policy_mapping_fn=lambda aid, ep, **kw: aid)
           .training(lr=2e-3, gamma=0.5, train_batch_size=64, model={"fcnet_hiddens": [32]})
           .debugging(seed=0))
    cfg.num_steps_sampled_before_learning_starts = 200
    cfg.target_network_update_freq = 100
    cfg.epsilon = [(0, 1.0), (2000, 0.02)]
    cfg.rollout_fragment_length = 10
    algo = cfg.build()
    best = {}
    for _ in range(120):
        res = algo.train()
        for k, v in res.get("module_episode_returns_mean", {}).items():
            best[k] = max(best.get(k, 0.0), v)
        if best and algo.total_env_steps > 2000 and min(best.values()) > 4.0:
            break
    algo.stop()
    assert any(k.endswith("/loss") for k in res["learners"])
    assert min(best.get("p1", 0), best.get("p2", 0)) > 3.5, best
