"""Connector pieces of the reference's pipelines (rllib/connectors/{common,env_to_module,
module_to_env,learner}/) on ray_amd's lock-step batches, and in a training run."""
import numpy as np
import pytest
import torch

import ray_amd as ray
from ray_amd.rllib.connectors.env_to_module import (AddObservationsFromEpisodesToBatch,
                                                    BatchIndividualItems, EnvToModulePipeline,
                                                    NumpyToTensor)
from ray_amd.rllib.connectors.learner import GeneralAdvantageEstimation
from ray_amd.rllib.connectors.module_to_env import (GetActions, ModuleToEnvPipeline,
                                                    RemoveSingleTsTimeRankFromBatch,
                                                    TensorToNumpy, UnBatchToIndividualItems)


def test_pieces_on_batches():
    b = BatchIndividualItems()(batch={"obs": [np.zeros(3), np.ones(3)]})
    assert b["obs"].shape == (2, 3)
    t = NumpyToTensor()(batch={"obs": np.ones((2, 3), np.float32), "name": ["a", "b"]})
    assert isinstance(t["obs"], torch.Tensor) and t["name"] == ["a", "b"]
    back = TensorToNumpy()(batch=t)
    assert isinstance(back["obs"], np.ndarray)
    m2e = ModuleToEnvPipeline(connectors=[GetActions(), TensorToNumpy(),
                                          UnBatchToIndividualItems()])
    out = m2e(batch={"action_dist_inputs": np.array([[0.0, 9.0], [9.0, 0.0]], np.float32)},
              explore=False)
    assert [int(a) for a in out["actions_for_env"]] == [1, 0]
    assert out["action_logp"].shape == (2,)
    r = RemoveSingleTsTimeRankFromBatch()(batch={"vf_preds": np.zeros((4, 1)),
                                                 "obs": np.zeros((4, 1))})
    assert r["vf_preds"].shape == (4,) and r["obs"].shape == (4, 1)

    class Ep:
        def __init__(self, v):
            self.observations = [np.full(2, v)]

    e2m = EnvToModulePipeline(connectors=[AddObservationsFromEpisodesToBatch()])
    assert e2m(batch={}, episodes=[Ep(1.0), Ep(2.0)])["obs"][:, 0].tolist() == [1.0, 2.0]


def test_gae_piece_matches_recursion():
    rng = np.random.default_rng(0)
    T, B = 6, 3
    r, v = rng.normal(size=(T, B)), rng.normal(size=(T, B))
    d = (rng.random((T, B)) < 0.2).astype(np.float64)
    out = GeneralAdvantageEstimation(gamma=0.97, lambda_=0.9)(
        batch={"rewards": r, "vf_preds": v, "terminateds": d})
    adv = np.zeros((T, B))
    for b_ in range(B):
        acc = 0.0
        for t in reversed(range(T)):
            nv = 0.0 if t == T - 1 else v[t + 1, b_]
            delta = r[t, b_] + 0.97 * nv * (1 - d[t, b_]) - v[t, b_]
            acc = delta + 0.97 * 0.9 * (1 - d[t, b_]) * acc
            adv[t, b_] = acc
    assert np.allclose(out["advantages"], adv, atol=1e-5)
    assert np.allclose(out["value_targets"], adv + v, atol=1e-5)


def test_pipeline_pieces_in_training():
    from ray_amd.rllib.algorithms import PPOConfig

    started = not ray.is_initialized()
    if started:
        ray.init(num_cpus=2)
    try:
        cfg = (PPOConfig().environment("CartPole-v1")
               .env_runners(num_env_runners=0, rollout_fragment_length=64,
                            env_to_module_connector=lambda *a: [
                                AddObservationsFromEpisodesToBatch(), BatchIndividualItems()],
                            module_to_env_connector=lambda *a: [UnBatchToIndividualItems()])
               .training(train_batch_size=128, minibatch_size=64, num_epochs=1))
        algo = cfg.build()
        res = algo.train()
        assert res["num_env_steps_sampled_lifetime"] >= 128
        algo.stop()
    finally:
        if started:
            ray.shutdown()


def test_old_stack_models_and_evaluation_pieces():
    from ray_amd.rllib.env import spaces
    from ray_amd.rllib.evaluation import (MultiAgentSampleBatchBuilder, RolloutWorker,
                                          SampleBatchBuilder, collect_metrics)
    from ray_amd.rllib.models import ModelCatalog
    from ray_amd.rllib.models.torch.torch_action_dist import (TorchCategorical,
                                                              TorchDiagGaussian)

    sp = spaces.Tuple((spaces.Discrete(2), spaces.Box(-1, 1, (3,))))
    p = ModelCatalog.get_preprocessor_for_space(sp)
    assert p.shape == (5,) and p.transform((1, np.ones(3))).tolist() == [0, 1, 1, 1, 1]
    oh = ModelCatalog.get_preprocessor_for_space(spaces.MultiDiscrete([2, 3]))
    assert oh.transform(np.array([1, 2])).tolist() == [0, 1, 0, 0, 1]
    d = TorchCategorical(torch.tensor([[0.0, 50.0]]))
    assert int(d.deterministic_sample()) == 1 and float(d.entropy()) < 1e-6
    g1, g2 = TorchDiagGaussian(torch.zeros(1, 2)), TorchDiagGaussian(torch.tensor([[1.0, 0.0]]))
    assert float(g1.kl(g2)) == pytest.approx(0.5)
    assert TorchDiagGaussian.required_model_output_shape(spaces.Box(-1, 1, (3,))) == 6
    mb = MultiAgentSampleBatchBuilder()
    mb.add_values("a0", "p0", obs=1, rewards=3.0)
    mb.add_values("a1", "p1", obs=2, rewards=-2.0)
    ma = mb.build_and_reset()
    assert set(ma.policy_batches) == {"p0", "p1"}
    sb = SampleBatchBuilder()
    sb.add_batch({"x": np.arange(3)})
    assert sb.build_and_reset()["x"].tolist() == [0, 1, 2]
    w = RolloutWorker({"env": "CartPole-v1", "num_envs_per_env_runner": 2,
                       "module_kind": "actor_critic", "rollout_fragment_length": 300})
    w.sample()
    m = collect_metrics([w])
    assert m["episodes_this_iter"] >= 1 and m["episode_reward_mean"] > 0


def test_old_stack_exploration():
    from ray_amd.rllib.env import spaces
    from ray_amd.rllib.models.action_dist import TorchCategorical, TorchDeterministic
    from ray_amd.rllib.utils.exploration import (EpsilonGreedy, GaussianNoise,
                                                 OrnsteinUhlenbeckNoise, ParameterNoise,
                                                 PerWorkerEpsilonGreedy, SoftQ,
                                                 StochasticSampling)

    q = torch.tensor([[0.0, 5.0, 1.0]] * 400)
    eg = EpsilonGreedy(spaces.Discrete(3), initial_epsilon=1.0, final_epsilon=0.0,
                       epsilon_timesteps=100, seed=0)
    a0, _ = eg.get_exploration_action(action_distribution=TorchCategorical(q), timestep=0)
    assert (a0 != 1).float().mean() > 0.5  # epsilon 1: mostly random
    a1, _ = eg.get_exploration_action(action_distribution=TorchCategorical(q), timestep=200)
    assert bool((a1 == 1).all())  # annealed to 0: greedy
    assert eg.get_state()["cur_epsilon"] == 0.0
    pw = [PerWorkerEpsilonGreedy(spaces.Discrete(3), num_workers=4, worker_index=i)
          for i in range(5)]
    eps = [p.epsilon(0) for p in pw]
    assert eps[0] == 0.0 and eps[1] == pytest.approx(0.4) and eps[1] > eps[2] > eps[4]
    ss = StochasticSampling(spaces.Discrete(3))
    a, lp = ss.get_exploration_action(action_distribution=TorchCategorical(q[:4]),
                                      timestep=1, explore=False)
    assert a.tolist() == [1, 1, 1, 1]
    sq, _ = SoftQ(spaces.Discrete(3), temperature=100.0).get_exploration_action(
        action_distribution=TorchCategorical(q), timestep=1)
    assert len(set(sq.tolist())) == 3  # high temperature: near uniform
    box = spaces.Box(-1.0, 1.0, (2,))
    gn = GaussianNoise(box, random_timesteps=0, stddev=0.5, initial_scale=1.0, seed=0)
    det = TorchDeterministic(torch.zeros(500, 2))
    ga, _ = gn.get_exploration_action(action_distribution=det, timestep=5)
    assert float(ga.std()) > 0.2 and float(ga.abs().max()) <= 1.0
    ou = OrnsteinUhlenbeckNoise(box, random_timesteps=0, seed=0)
    o1, _ = ou.get_exploration_action(action_distribution=TorchDeterministic(torch.zeros(1, 2)),
                                      timestep=5)
    assert ou.get_state()["ou_state"] is not None
    model = torch.nn.Linear(2, 2)
    w0 = model.weight.detach().clone()
    pn = ParameterNoise(box, model=model, initial_stddev=0.5)
    pn.on_episode_start()
    assert not torch.equal(model.weight, w0)
    pn.on_episode_end()
    assert torch.allclose(model.weight, w0)


def test_sample_batch_and_multi_agent_env_helpers():
    from ray_amd.rllib.env import spaces
    from ray_amd.rllib.env.multi_agent_env import make_multi_agent
    from ray_amd.rllib.env.envs import CartPoleEnv
    from ray_amd.rllib.policy_sample_batch import MultiAgentBatch, SampleBatch

    b = SampleBatch({"obs": np.arange(12.0).reshape(6, 2), "terminateds": [0, 0, 1, 0, 0, 1],
                     "eps_id": [0, 0, 0, 1, 1, 1]})
    assert b.is_terminated_or_truncated() and not b.is_single_trajectory()
    assert b.slice(0, 3).is_single_trajectory()
    one = b.get_single_step_input_dict()
    assert len(one) == 1 and one["obs"][0].tolist() == [10.0, 11.0]
    b.compress(columns=("obs",))
    b.decompress_if_needed(columns=("obs",))
    assert b["obs"].shape == (6, 2) and b["obs"][5, 1] == 11.0
    b.set_training(True)
    assert b.is_training()
    b.set_get_interceptor(lambda v: np.asarray(v) * 0)
    assert float(b["obs"].sum()) == 0.0
    s = SampleBatch({"x": np.arange(5), "seq_lens": np.array([2, 3])})
    s.zero_pad(4)
    assert s["x"].tolist() == [0, 1, 0, 0, 2, 3, 4, 0] and len(s) == 8
    ma = MultiAgentBatch({"p": SampleBatch({"x": np.arange(10)})}, 10)
    parts = ma.timeslices(4)
    assert [len(p) for p in parts] == [4, 4, 2]
    assert len(MultiAgentBatch.concat_samples(parts)) == 10
    MA = make_multi_agent(lambda cfg: CartPoleEnv(cfg))
    env = MA({"num_agents": 2})
    acts = env.action_space_sample()
    assert set(acts) == {0, 1} and env.action_space_contains(acts)
    obs, _ = env.reset(seed=0)
    assert env.observation_space_contains(obs)
    assert set(env.with_agent_groups({"g": [0, 1]}).reset(seed=0)[0]) == {"g"}
    base = env.to_base_env()
    o, *_ = base.poll()
    assert set(o[0]) == {0, 1}


def test_custom_searcher_and_scheduler_hooks(tmp_path):
    from ray_amd.tune.schedulers import FIFOScheduler
    from ray_amd.tune.search import Searcher

    class Grid(Searcher):
        def __init__(self):
            super().__init__(metric="m", mode="max")
            self.seen = []
            self.i = 0

        def suggest(self, trial_id):
            self.i += 1
            return {"x": self.i}

        def add_evaluated_point(self, parameters, value, **kw):
            self.seen.append((parameters["x"], value))

    g = Grid()
    g.add_evaluated_point({"x": 7}, 1.5)
    g.suggest("t1")
    g.save_to_dir(str(tmp_path))
    h = Grid()
    h.restore_from_dir(str(tmp_path))
    assert h.seen == [(7, 1.5)] and h.i == 1 and h.metric == "m"
    sch = FIFOScheduler()
    assert sch.supports_buffered_results and "FIFOScheduler" in sch.debug_string()
    sch.metric = "loss"
    sch.save(str(tmp_path / "s.pkl"))
    s2 = FIFOScheduler()
    s2.restore(str(tmp_path / "s.pkl"))
    assert s2.metric == "loss"


def test_rl_module_checkpoints_and_multi_module(tmp_path):
    from ray_amd.rllib.core.rl_module import MultiRLModule, RLModule, TorchRLModule
    from ray_amd.rllib.env import spaces
    from ray_amd.rllib.models.action_dist import TorchCategorical

    obs_sp, act_sp = spaces.Box(-1, 1, (4,)), spaces.Discrete(2)
    m = RLModule(obs_sp, act_sp, {"fcnet_hiddens": [16]})
    path = m.save_to_checkpoint(str(tmp_path / "m"))
    m2 = RLModule.from_checkpoint(path)
    x = torch.randn(3, 4)
    with torch.no_grad():
        a = m.forward_inference({"obs": x})["action_dist_inputs"]
        b = m2.forward_inference({"obs": x})["action_dist_inputs"]
    assert torch.allclose(a, b)
    assert m.get_inference_action_dist_cls() is TorchCategorical and m.unwrapped() is m

    class Tiny(TorchRLModule):
        def setup(self):
            self.lin = torch.nn.Linear(4, 2)

        def _forward(self, batch, **kw):
            return {"action_dist_inputs": self.lin(batch["obs"])}

    t = Tiny(obs_sp, act_sp, model_config={"k": 1})
    mm = t.as_multi_agent()
    mm.add_module("other", RLModule(obs_sp, act_sp, {"fcnet_hiddens": [8]}))
    assert set(mm.keys()) == {"default_policy", "other"}
    out = mm.forward_inference({"default_policy": {"obs": x}})
    assert out["default_policy"]["action_dist_inputs"].shape == (3, 2)
    mp = mm.save_to_checkpoint(str(tmp_path / "mm"))
    back = MultiRLModule.from_checkpoint(mp)
    assert set(back.keys()) == {"default_policy", "other"}
    with torch.no_grad():
        assert torch.allclose(back["default_policy"].lin.weight, t.lin.weight)
    mm.remove_module("other")
    assert list(mm.keys()) == ["default_policy"]


def test_old_stack_policy_surface(tmp_path):
    from ray_amd.rllib.env import spaces
    from ray_amd.rllib.policy import Policy, TorchPolicy
    from ray_amd.rllib.policy_sample_batch import SampleBatch
    from ray_amd.rllib.utils.replay_buffers import ReplayBuffer

    model = torch.nn.Linear(3, 2)

    def loss_fn(policy, m, batch):
        lp = policy.action_log_prob(batch["obs"].float(), batch["actions"])
        return -(lp * batch["rewards"].float()).mean()

    pol = TorchPolicy(spaces.Box(-1, 1, (3,)), spaces.Discrete(2), {"lr": 0.1,
                                                                    "train_batch_size": 8},
                      model=model, loss_fn=loss_fn)
    obs = np.random.default_rng(0).normal(size=(8, 3)).astype(np.float32)
    acts, _, extra = pol.compute_actions_from_input_dict({"obs": obs}, explore=False)
    assert acts.shape == (8,)
    ll = pol.compute_log_likelihoods(acts, obs)
    assert np.all(ll <= 0) and np.allclose(ll, extra["action_logp"] * 0 + ll)
    batch = SampleBatch({"obs": obs, "actions": acts, "rewards": np.ones(8, np.float32)})
    w0 = model.weight.detach().clone()
    grads, info = pol.compute_gradients(batch)
    pol.apply_gradients(grads)
    assert not torch.allclose(model.weight, w0) and "total_loss" in info["learner_stats"]
    assert pol.load_batch_into_buffer(batch) == 8
    assert pol.get_num_samples_loaded_into_buffer() == 8
    assert "learner_stats" in pol.learn_on_loaded_batch(0)
    rb = ReplayBuffer(100)
    rb.add({"obs": obs, "actions": acts, "rewards": np.ones(8, np.float32)})
    assert "learner_stats" in pol.learn_on_batch_from_replay_buffer(rb, "default_policy")
    pol.export_model(str(tmp_path / "exp"))
    assert (tmp_path / "exp" / "model.pt").exists()
    assert pol.apply(lambda p, k: k + 1, 1) == 2 and pol.postprocess_trajectory(batch) is batch


def test_dag_node_helpers():
    import ray_amd as ray
    from ray_amd.dag import DAGNode, InputNode

    started = not ray.is_initialized()
    if started:
        ray.init(num_cpus=2)
    try:
        @ray.remote
        def inc(x):
            return x + 1

        with InputNode() as inp:
            dag = inc.bind(inc.bind(inp))
        assert ray.get(dag.execute(1)) == 3
        refs = dag.get_object_refs_from_last_execute()
        assert len(refs) >= 2 and dag.get_stable_uuid() in refs
        dag.clear_cache()
        assert dag.get_object_refs_from_last_execute() == {}
        seen = []
        dag.apply_recursive(lambda n: seen.append(type(n).__name__) or n)
        assert seen[-1] == type(dag).__name__ and len(seen) == 3
        out = dag.apply_functional([1, (2, {"a": 3})], lambda v: isinstance(v, int),
                                   lambda v: v * 10)
        assert out == [10, (20, {"a": 30})]
        assert isinstance(dag, DAGNode)
    finally:
        if started:
            ray.shutdown()


def test_multi_agent_episode_turn_based_credit():
    from ray_amd.rllib.env.multi_agent_episode import MultiAgentEpisode

    ep = MultiAgentEpisode(agent_to_module_mapping_fn=lambda aid, e: f"m_{aid}")
    ep.add_env_reset(observations={"a": 0})
    # turn-based: a acts, b observes next; a's reward arrives later
    ep.add_env_step({"b": 10}, {"a": 1}, {"a": 0.5})
    assert ep.get_agents_to_act() == {"b"} and len(ep.agent_episodes["a"]) == 0
    ep.add_env_step({"a": 1}, {"b": 2}, {"a": 1.0, "b": 0.0})
    assert len(ep.agent_episodes["a"]) == 1
    assert ep.agent_episodes["a"].rewards == [1.5]  # hanging reward credited on observation
    nxt = ep.cut()
    ep.add_env_step({"b": 11}, {"a": 0}, {"b": 2.0},
                    terminateds={"__all__": True})
    assert ep.is_done and ep.agent_episodes["b"].rewards == [2.0]
    assert ep.get_return() == pytest.approx(3.5)
    ma = ep.get_sample_batch()
    assert set(ma.policy_batches) == {"m_a", "m_b"}
    assert ep.module_for("a") == "m_a" and nxt.id_ == ep.id_
    back = MultiAgentEpisode.from_state(ep.get_state())
    assert back.get_return() == pytest.approx(3.5) and back.is_done
