"""Classic RLlib env / policy APIs (reference: rllib/env/vector_env.py,
rllib/env/external_env.py, rllib/policy/policy.py; tests modelled on
rllib/env/tests/test_external_env.py and rllib/policy/tests/test_policy.py)."""
import numpy as np
import pytest
import torch

import ray_amd as ray
from ray_amd.rllib import ExternalEnv, Policy, TorchPolicy, VectorEnv
from ray_amd.rllib.algorithms.ppo import PPOConfig
from ray_amd.rllib.env import spaces
from ray_amd.rllib.env.envs import CartPoleEnv, make_env


@pytest.fixture(scope="module", autouse=True)
def cluster():
    ray.init(num_cpus=4)
    yield
    ray.shutdown()


class _Flaky(CartPoleEnv):
    def step(self, a):
        if getattr(self, "boom", False):
            raise RuntimeError("simulator crashed")
        return super().step(a)


def test_vectorize_reset_step_and_restart():
    made = []

    def mk(i):
        e = _Flaky({"seed": i})
        made.append(e)
        return e

    v = VectorEnv.vectorize_gym_envs(make_env=mk, num_envs=3,
                                     restart_failed_sub_environments=True)
    obs, infos = v.vector_reset(seeds=[0, 1, 2])
    assert v.num_envs == 3 and len(obs) == 3 and obs[0].shape == (4,)
    v.envs[1].boom = True
    o, r, te, tr, inf = v.vector_step([0, 1, 0])
    assert tr[1] and "env_error" in inf[1] and not tr[0]
    v.reset_at(1)  # the failed slot is rebuilt
    assert len(made) == 4 and v.envs[1] is made[-1]
    strict = VectorEnv.vectorize_gym_envs(existing_envs=[_Flaky()], num_envs=1)
    strict.vector_reset()
    strict.envs[0].boom = True
    with pytest.raises(RuntimeError, match="crashed"):
        strict.vector_step([0])


class CartPoleExternal(ExternalEnv):
    """CartPole driven from its own thread through get_action / log_returns."""

    def __init__(self, config=None):
        self.sim = CartPoleEnv(config or {})
        super().__init__(self.sim.action_space, self.sim.observation_space)

    def run(self):
        while True:
            eid = self.start_episode()
            obs, _ = self.sim.reset()
            done = False
            while not done:
                a = self.get_action(eid, obs)
                obs, r, te, tr, _ = self.sim.step(a)
                self.log_returns(eid, r)
                done = te or tr
            self.end_episode(eid, obs)


def test_external_env_adapter_protocol():
    env = make_env(CartPoleExternal, {"seed": 3})
    obs, _ = env.reset()
    assert obs.shape == (4,)
    total, steps = 0.0, 0
    while True:
        obs, r, done, trunc, _ = env.step(steps % 2)
        total += r
        steps += 1
        if done:
            break
    assert total == steps  # +1 per step, all logged returns delivered
    obs2, _ = env.reset()  # next episode
    assert obs2.shape == (4,)
    with pytest.raises(NotImplementedError, match="offline"):
        env.ext.log_action("x", obs2, 0)


def test_ppo_trains_on_external_env():
    algo = (PPOConfig().environment(CartPoleExternal)
            .env_runners(num_env_runners=0, num_envs_per_env_runner=2)
            .training(train_batch_size=400, minibatch_size=100, num_epochs=2)
            .debugging(seed=0)).build()
    r = algo.train()
    assert r["num_env_steps_sampled_this_iter"] >= 400 and r["env_runners"]["num_episodes"] > 0
    assert r["env_runners"]["episode_return_mean"] > 0
    algo.stop()


def test_env_runner_flattens_vector_env():
    def creator(cfg):
        return VectorEnv.vectorize_gym_envs(make_env=lambda i: CartPoleEnv({"seed": i}),
                                            num_envs=3)

    algo = (PPOConfig().environment(creator)
            .env_runners(num_env_runners=0, num_envs_per_env_runner=2)
            .training(train_batch_size=300, minibatch_size=100, num_epochs=1)).build()
    assert len(algo.local_runner.envs) == 6
    algo.train()
    assert isinstance(algo.get_policy(), Policy)
    algo.stop()


def test_torch_policy_actions_learning_and_checkpoint(tmp_path):
    torch.manual_seed(0)
    obs_space = spaces.Box(-1.0, 1.0, (3,), np.float32)
    act_space = spaces.Discrete(2)
    model = torch.nn.Linear(3, 2)

    def imitation(policy, model, batch):  # learn action = (obs[0] > 0)
        return -policy.action_log_prob(batch["obs"].float(), batch["actions"]).mean()

    p = TorchPolicy(obs_space, act_space, {"lr": 0.1}, model=model, loss_fn=imitation)
    x = np.random.default_rng(0).uniform(-1, 1, (256, 3)).astype(np.float32)
    acts, st, extra = p.compute_actions(x)
    assert acts.shape == (256,) and st == [] and extra["action_logp"].shape == (256,)
    y = (x[:, 0] > 0).astype(np.int64)
    first = p.learn_on_batch({"obs": x, "actions": y})["learner_stats"]["total_loss"]
    for _ in range(50):
        last = p.learn_on_batch({"obs": x, "actions": y})["learner_stats"]["total_loss"]
    assert last < first * 0.6
    greedy, _, _ = p.compute_actions(x, explore=False)
    assert (greedy == y).mean() > 0.9
    a, _, _ = p.compute_single_action(x[0], explore=False)
    assert a == greedy[0]
    p2 = TorchPolicy(obs_space, act_space, model=torch.nn.Linear(3, 2))
    p2.set_state(p.get_state())
    np.testing.assert_array_equal(p2.compute_actions(x, explore=False)[0], greedy)
    p.export_checkpoint(str(tmp_path / "pc"))
    with pytest.raises(TypeError, match="model"):
        Policy.from_checkpoint(str(tmp_path / "pc"))


def test_plain_policy_subclass_checkpoint(tmp_path):
    class Const(Policy):
        def __init__(self, obs, act, cfg=None):
            super().__init__(obs, act, cfg)
            self.w = {"c": 1}

        def compute_actions(self, obs_batch, state_batches=None, **kw):
            return np.full(len(obs_batch), self.w["c"]), [], {}

        def get_weights(self):
            return dict(self.w)

        def set_weights(self, w):
            self.w = dict(w)

    p = Const(spaces.Box(-1.0, 1.0, (2,), np.float32), spaces.Discrete(3))
    p.set_weights({"c": 2})
    p.export_checkpoint(str(tmp_path / "c"))
    q = Policy.from_checkpoint(str(tmp_path / "c"))
    assert isinstance(q, Const) and q.compute_single_action(np.zeros(2))[0] == 2
