"""The RLlib learner pipeline and LearnerGroup (modelled on rllib/core/learner/tests/
test_learner.py, test_learner_group.py and rllib/algorithms/tests/test_algorithm.py's
add/remove module cases): compute_losses -> compute_gradients -> postprocess_gradients
-> apply_gradients behind update_from_batch / update_from_episodes, save_state /
load_state, foreach_learner, off-policy algorithms on 2 gloo learners with identical
weights, a postprocess_gradients override, and a self-play module added mid-training."""

import numpy as np
import pytest
import torch

import ray_amd as ray
from ray_amd.rllib.algorithms.dqn import DQNConfig, DQNLearner
from ray_amd.rllib.algorithms.ppo import PPOConfig
from ray_amd.rllib.algorithms.sac import SACConfig, SACLearner
from ray_amd.rllib.core.learner import Learner, LearnerGroup
from ray_amd.rllib.env import make_env


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6)
    yield
    ray.shutdown()


def _cartpole_batch(n=64, seed=0):
    rng = np.random.default_rng(seed)
    return {"obs": rng.standard_normal((n, 4)).astype(np.float32),
            "next_obs": rng.standard_normal((n, 4)).astype(np.float32),
            "actions": rng.integers(0, 2, n), "rewards": np.ones(n, np.float32),
            "terminateds": (rng.random(n) < 0.05).astype(np.float32)}


def _dqn_cfg(**kw):
    c = {"model": {"fcnet_hiddens": [32]}, "lr": 1e-3, "gamma": 0.99, "double_q": True,
         "dueling": True, "grad_clip": 10.0, "num_gpus_per_learner": 0, "seed": 0}
    c.update(kw)
    return c


def test_learner_pipeline_hooks_called_in_order_and_state_roundtrip(tmp_path):
    env = make_env("CartPole-v1", {})
    calls = []

    class Traced(DQNLearner):
        def compute_losses(self, *, fwd_out, batch):
            calls.append("losses")
            return super().compute_losses(fwd_out=fwd_out, batch=batch)

        def compute_gradients(self, loss_per_module, **kw):
            calls.append("gradients")
            return super().compute_gradients(loss_per_module, **kw)

        def postprocess_gradients(self, g):
            calls.append("postprocess")
            return super().postprocess_gradients(g)

        def apply_gradients(self, g):
            calls.append("apply")
            return super().apply_gradients(g)

    lr = Traced(_dqn_cfg(), env.observation_space, env.action_space)
    res = lr.update_from_batch(_cartpole_batch())
    assert calls == ["losses", "gradients", "postprocess", "apply"]
    assert res["td_error"].shape == (64,) and np.isfinite(res["loss"])
    # minibatches over epochs: per-row outputs still cover the whole batch
    res = lr.update_from_batch(_cartpole_batch(64, 1), num_epochs=2, minibatch_size=16,
                               shuffle_batch_per_epoch=True)
    assert res["td_error"].shape == (64,)
    path = lr.save_state(str(tmp_path / "ckpt"))
    w0 = {k: v.clone() for k, v in lr.get_weights().items()}
    lr.update_from_batch(_cartpole_batch(64, 2))
    assert any(not torch.equal(w0[k], v) for k, v in lr.get_weights().items())
    lr2 = DQNLearner(_dqn_cfg(seed=5), env.observation_space, env.action_space)
    lr2.load_state(path)
    assert all(torch.equal(w0[k], v) for k, v in lr2.get_weights().items())
    assert lr2.get_optimizer().state_dict()["state"]  # Adam moments restored too


def test_update_from_episodes(tmp_path):
    from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode

    env = make_env("CartPole-v1", {})
    eps = []
    for s in range(3):
        ep = SingleAgentEpisode()
        o, _ = env.reset(seed=s)
        ep.add_env_reset(o)
        for t in range(10):
            a = t % 2
            o, r, te, tr, _ = env.step(a)
            ep.add_env_step(o, a, r, terminated=te, truncated=tr)
            if te or tr:
                break
        eps.append(ep)
    lr = DQNLearner(_dqn_cfg(), env.observation_space, env.action_space)
    res = lr.update_from_episodes(eps)
    assert res["td_error"].shape[0] == sum(len(e.get_actions()) for e in eps)


def test_postprocess_gradients_override_freezes_training():
    env = make_env("CartPole-v1", {})

    class NoGrad(DQNLearner):
        def postprocess_gradients(self, gradients_dict):
            return {k: torch.zeros_like(g) for k, g in gradients_dict.items()}

    lr = NoGrad(_dqn_cfg(), env.observation_space, env.action_space)
    w0 = {k: v.clone() for k, v in lr.get_weights().items()}
    for i in range(3):
        lr.update_from_batch(_cartpole_batch(32, i))
    # Adam with all-zero gradients leaves the weights unchanged
    assert all(torch.equal(w0[k], v) for k, v in lr.get_weights().items())


def test_ppo_learner_postprocess_override_takes_the_eager_path():
    """An overridden gradient hook on the fused PPO Learner switches it to the eager
    pipeline (the captured fused step would bypass the hook)."""
    env = make_env("CartPole-v1", {})
    seen = []

    class Scaled(Learner):
        def postprocess_gradients(self, g):
            seen.append(len(g))
            return {k: v * 0.0 for k, v in g.items()}

    cfg = {"model": {"fcnet_hiddens": [16]}, "num_gpus_per_learner": 0, "seed": 0, "lr": 1e-2,
           "num_epochs": 1, "minibatch_size": 32, "train_batch_size": 64}
    lr = Scaled(cfg, env.observation_space, env.action_space)
    assert lr._generic
    T, B = 16, 4
    rng = np.random.default_rng(0)
    batch = {"obs": rng.standard_normal((T, B, 4)).astype(np.float32),
             "actions": rng.integers(0, 2, (T, B)), "rewards": np.ones((T, B), np.float32),
             "terminateds": np.zeros((T, B), np.float32),
             "truncateds": np.zeros((T, B), np.float32),
             "action_logp": np.full((T, B), np.log(0.5), np.float32),
             "action_dist_inputs": np.zeros((T, B, 2), np.float32),
             "bootstrap_obs": rng.standard_normal((B, 4)).astype(np.float32)}
    w0 = {k: v.clone() for k, v in lr.get_weights().items()}
    lr.update_from_batch(batch)
    assert seen  # the hook ran
    assert all(torch.equal(w0[k], v) for k, v in lr.get_weights().items())


def _weights_equal_across(group):
    ws = group.foreach_learner(lambda lr: {k: v.detach().cpu().numpy().copy()
                                           for k, v in lr.module.state_dict().items()})
    assert len(ws) == 2
    for k in ws[0]:
        np.testing.assert_array_equal(ws[0][k], ws[1][k], err_msg=k)
    return ws


def test_dqn_two_gloo_learners_identical_weights(cluster):
    cfg = (DQNConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=0)
           .learners(num_learners=2, num_gpus_per_learner=0)
           .training(train_batch_size=32, num_steps_sampled_before_learning_starts=64,
                     model={"fcnet_hiddens": [32]}, learner_backend="gloo")
           .debugging(seed=0))
    cfg.rollout_fragment_length = 64
    algo = cfg.build()
    try:
        assert isinstance(algo.learner_group, LearnerGroup) and algo.learner_group.remote
        w_init = algo.get_weights()
        for _ in range(3):
            res = algo.train()
        assert np.isfinite(res["learners"]["loss"])
        ws = _weights_equal_across(algo.learner_group)
        # the learners trained (not a no-op)
        assert any(not np.array_equal(np.asarray(w_init[k]), ws[0]["q." + k])
                   for k in w_init)
    finally:
        algo.stop()


def test_sac_two_gloo_learners_identical_weights(cluster):
    cfg = (SACConfig().environment("Pendulum-v1")
           .env_runners(num_env_runners=0)
           .learners(num_learners=2, num_gpus_per_learner=0)
           .training(train_batch_size=32, num_steps_sampled_before_learning_starts=64,
                     model={"fcnet_hiddens": [32, 32]}, learner_backend="gloo")
           .debugging(seed=0))
    cfg.rollout_fragment_length = 64
    algo = cfg.build()
    try:
        for _ in range(3):
            res = algo.train()
        assert np.isfinite(res["learners"]["critic_loss"])
        ws = _weights_equal_across(algo.learner_group)
        assert "log_alpha" in ws[0]
        a = algo.compute_single_action(np.zeros(3, np.float32))
        assert a.shape == (1,)
    finally:
        algo.stop()


def test_self_play_add_module_mid_training(cluster):
    """League / self-play: train "main", then add a frozen snapshot "main_v1" as the
    opponent of agent 1 mid-training; only "main" keeps learning."""
    cfg = (PPOConfig().environment("MultiAgentCartPole", env_config={"num_agents": 2})
           .env_runners(num_env_runners=1, num_envs_per_env_runner=2)
           .multi_agent(policies={"main"}, policy_mapping_fn=lambda aid, ep, **kw: "main")
           .training(train_batch_size=400, minibatch_size=100, num_epochs=2, lr=1e-3,
                     model={"fcnet_hiddens": [32]})
           .debugging(seed=0))
    algo = cfg.build()
    try:
        algo.train()
        snap = {k: np.asarray(v).copy() for k, v in algo.get_weights()["main"].items()}
        ids = algo.add_module(
            "main_v1", weights=snap,
            new_agent_to_module_mapping_fn=lambda aid, ep, **kw: "main" if aid == 0
            else "main_v1",
            new_should_module_be_updated=["main"])
        assert set(ids) == {"main", "main_v1"}
        assert algo.config.policies_to_train == ["main"]
        for _ in range(2):
            res = algo.train()
        w = algo.get_weights()
        for k, v in w["main_v1"].items():  # frozen opponent: unchanged
            np.testing.assert_array_equal(np.asarray(v), snap[k])
        assert any(not np.array_equal(np.asarray(w["main"][k]), snap[k]) for k in snap)
        assert set(res["module_episode_returns_mean"]) == {"main", "main_v1"}
        # the runner plays the snapshot with the snapshot's weights
        got = algo.env_runner_group.foreach_env_runner(
            lambda r: {k: v.numpy().copy() for k, v in r.modules["main_v1"].state_dict()
                       .items()})[0]
        for k, v in got.items():
            np.testing.assert_array_equal(v, snap[k])
        algo.remove_module("main_v1",
                           new_agent_to_module_mapping_fn=lambda aid, ep, **kw: "main")
        res = algo.train()
        assert set(algo.get_weights()) == {"main"}
    finally:
        algo.stop()


def test_two_gloo_learners_add_module_and_restore_optimizer_state(cluster):
    """Learner / LearnerGroup module-set API (reference: learner.py:607,696,714,821,845,
    1308,1316; learner_group.py:494,520): a module added mid-training trains with
    identical weights on both ranks, and a second group restored from the first's module
    + optimizer state takes the next update bit-exactly like the first."""
    env = make_env("CartPole-v1", {})
    cfg = _dqn_cfg(num_learners=2, learner_backend="gloo")

    def group():
        return LearnerGroup(cfg, env.observation_space, env.action_space,
                            learner_class=DQNLearner)

    g = group()
    try:
        g.update_from_batch(_cartpole_batch(64, 0), minibatch_size=16)
        ids = g.add_module(module_id="opp", module_spec=(env.observation_space,
                                                         env.action_space),
                           config_overrides={"lr": 5e-3})
        assert ids == ["default_policy", "opp"]
        w_opp0 = g.get_module_state(["opp"])["opp"]
        for i in range(3):
            res = g.update_from_batch({"default_policy": _cartpole_batch(64, 10 + i),
                                       "opp": _cartpole_batch(48, 20 + i)},
                                      minibatch_size=16, shuffle_batch_per_epoch=True)
        assert "opp/loss" in res and np.isfinite(res["opp/loss"])
        both = g.foreach_learner(lambda lr: {m: {k: v.numpy().copy() for k, v in w.items()}
                                             for m, w in lr.get_module_state().items()})
        for m in ("default_policy", "opp"):
            for k in both[0][m]:
                np.testing.assert_array_equal(both[0][m][k], both[1][m][k], err_msg=f"{m}/{k}")
        assert any(not np.array_equal(np.asarray(w_opp0[k]), both[0]["opp"][k])
                   for k in w_opp0)
        lr_opp = g.foreach_learner(lambda lr: lr._module_learners()["opp"].get_optimizer()
                                   .param_groups[0]["lr"])
        assert lr_opp == [5e-3, 5e-3]  # config_overrides reached the module's optimizer

        # restore into a fresh group: module weights + optimizer moments
        ms, os_ = g.get_module_state(), g.get_optimizer_state()
        assert set(os_) == {"default_policy", "opp"} and os_["opp"]["opp/default"]["state"]
        h = group()
        try:
            h.add_module(module_id="opp", module_spec=(env.observation_space,
                                                       env.action_space),
                         config_overrides={"lr": 5e-3})
            h.set_module_state(ms)
            h.set_optimizer_state(os_)
            nb = {"default_policy": _cartpole_batch(64, 99), "opp": _cartpole_batch(48, 98)}
            g.update_from_batch(nb)
            h.update_from_batch(nb)
            a, b = g.get_module_state(), h.get_module_state()
            for m in a:
                for k in a[m]:
                    assert torch.equal(a[m][k], b[m][k]), f"{m}/{k}"
            # remove_module drops it from every learner
            assert h.remove_module("opp") == ["default_policy"]
            assert h.foreach_learner(lambda lr: lr.module_ids) == [["default_policy"]] * 2
        finally:
            h.shutdown()
    finally:
        g.shutdown()


def test_register_metrics_and_weights_only_state(tmp_path):
    env = make_env("CartPole-v1", {})
    lr = DQNLearner(_dqn_cfg(), env.observation_space, env.action_space)
    lr.add_module(module_id="b", module_spec=(env.observation_space, env.action_space))
    lr.register_metrics("b", {"my_metric": torch.tensor(2.5)})
    assert lr._module_learners()["b"].metrics["my_metric"] == 2.5
    res = lr.update_from_batch({"default_policy": _cartpole_batch(32, 0),
                                "b": _cartpole_batch(32, 1)})
    assert res["b/my_metric"] == 2.5
    path = lr.save_state(str(tmp_path / "s"))
    # loadable without unpickling code
    st = torch.load(str(tmp_path / "s" / "learner_state.pt"), weights_only=True)
    assert "b" in st["__modules__"]
    lr2 = DQNLearner(_dqn_cfg(seed=3), env.observation_space, env.action_space)
    lr2.add_module(module_id="b", module_spec=(env.observation_space, env.action_space))
    lr2.load_state(path)
    for m, w in lr.get_module_state().items():
        for k, v in w.items():
            assert torch.equal(v, lr2.get_module_state()[m][k])
    with pytest.raises(ValueError):
        lr.add_module(module_id="b")


def test_trainable_and_learner_surface():
    """Trainable-style Algorithm API and the remaining Learner / LearnerGroup methods
    (reference: algorithm.py step/cleanup/get_default_config/default_resource_request/
    merge_algorithm_configs; learner.py register_metric/compute_loss/apply/...;
    learner_group.py is_remote/get_stats/load_module_state)."""
    import os
    import tempfile

    import torch

    import ray_amd as ray
    from ray_amd.rllib.algorithms import PPO, PPOConfig
    from ray_amd.rllib.algorithms.algorithm import Algorithm

    cfg = PPO.get_default_config()
    assert isinstance(cfg, PPOConfig)
    merged = Algorithm.merge_algorithm_configs({"a": {"x": 1, "y": 2}, "b": 1},
                                               {"a": {"y": 3}, "c": 4})
    assert merged == {"a": {"x": 1, "y": 3}, "b": 1, "c": 4}
    with pytest.raises(ValueError):
        Algorithm.merge_algorithm_configs({"a": 1}, {"zz": 1}, _allow_unknown_configs=False)
    c = (PPOConfig().environment("CartPole-v1")
         .env_runners(num_env_runners=2, num_cpus_per_env_runner=1)
         .learners(num_learners=0, num_gpus_per_learner=0))
    pgf = PPO.default_resource_request(c)
    assert len(pgf.bundles) == 3 and pgf.bundles[1] == {"CPU": 1.0}
    assert "bundles" in PPO.resource_help(c)
    started = not ray.is_initialized()
    if started:
        ray.init(num_cpus=2)
    try:
        algo = (PPOConfig().environment("CartPole-v1")
                .env_runners(num_env_runners=0, num_envs_per_env_runner=2,
                             rollout_fragment_length=32)
                .training(train_batch_size=64, minibatch_size=32, num_epochs=1)
                .debugging(seed=0)).build()
        r = algo.step()
        assert r["training_iteration"] == 1
        algo.log_result(r)
        m = algo.get_auto_filled_metrics(time_this_iter=1.0)
        assert m["training_iteration"] == 1 and "pid" in m
        lg = algo.learner_group
        assert lg.is_remote is False and lg.get_stats()["num_learners"] == 1
        lr = lg.local
        assert lr.distributed is False
        assert lr.apply(lambda le, k: k + 1, 1) == 2
        mid = lr.module_ids[0]
        lr.register_metric(mid, "my_metric", 3.0)
        p0 = next(lr.module.parameters())
        assert isinstance(lr.get_param_ref(p0), str)
        opt = lr.get_optimizer()
        pd = dict(lr.module.named_parameters())
        assert lr.filter_param_dict_for_optimizer(pd, opt).keys() == pd.keys()
        assert lr.additional_update(timestep=0) == {m_: {} for m_ in lr.module_ids}
        with tempfile.TemporaryDirectory() as d:
            sd = lg.get_module_state()[mid]
            sd = {k: (v * 0 if torch.is_tensor(v) and v.is_floating_point() else v)
                  for k, v in sd.items()}
            os.makedirs(os.path.join(d, mid))
            torch.save(sd, os.path.join(d, mid, "module_state.pt"))
            lg.load_module_state(marl_module_ckpt_dir=d)
            assert all(float(v.abs().sum()) == 0 for v in lg.get_module_state()[mid].values()
                       if torch.is_tensor(v) and v.is_floating_point())
        algo.cleanup()
    finally:
        if started:
            ray.shutdown()
