"""RLlib extensibility: user RLModules (RLModuleSpec / TorchRLModule), Learner hooks
(compute_loss_for_module, configure_optimizers_for_module), SingleAgentEpisode +
EpisodeReplayBuffer (DQN from episodes, n-step) and the stateful LSTM module (reference:
rllib/core/rl_module/rl_module.py:58, core/learner/learner.py:435,948,
env/single_agent_episode.py:18, utils/replay_buffers/episode_replay_buffer.py:14,
core/models/torch/encoder.py:294)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

import ray_amd as ray
from ray_amd.rllib.algorithms.dqn import DQNConfig
from ray_amd.rllib.algorithms.ppo import PPOConfig
from ray_amd.rllib.core.columns import Columns
from ray_amd.rllib.core.learner import PPOTorchLearner
from ray_amd.rllib.core.rl_module import RLModuleSpec, TorchRLModule, ValueFunctionAPI
from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode
from ray_amd.rllib.utils.replay_buffers.episode_replay_buffer import EpisodeReplayBuffer


@pytest.fixture(scope="module")
def cluster():
    ray.init(num_cpus=6)
    yield
    ray.shutdown()


def test_single_agent_episode():
    e = SingleAgentEpisode("e1")
    e.add_env_reset(np.array([0.0]))
    for t in range(5):
        e.add_env_step(np.array([t + 1.0]), t % 2, 1.0, extra_model_outputs={"logp": -0.5})
    assert len(e) == 5 and e.get_return() == 5.0 and not e.is_done
    assert e.get_observations(-1)[0] == 5.0 and e.get_actions([0, 1]) == [0, 1]
    nxt = e.cut()
    assert nxt.id_ == "e1" and nxt.t_started == 5 and len(nxt) == 0
    nxt.add_env_step(np.array([6.0]), 1, 2.0, terminated=True)
    e.concat_episode(nxt)
    assert len(e) == 6 and e.is_terminated and e.get_return() == 7.0
    sl = e[2:4]
    assert len(sl) == 2 and sl.t_started == 2 and not sl.is_done
    assert len(e.get_extra_model_outputs("logp")) == 5
    s2 = SingleAgentEpisode.from_state(e.get_state())
    assert len(s2) == 6 and s2.is_terminated


def _ep(eid, rewards, terminated=True):
    e = SingleAgentEpisode(eid)
    e.add_env_reset(np.array([0.0], np.float32))
    for i, r in enumerate(rewards):
        e.add_env_step(np.array([i + 1.0], np.float32), i, r,
                       terminated=terminated and i == len(rewards) - 1)
    return e


def test_episode_replay_buffer_nstep_and_eviction():
    rb = EpisodeReplayBuffer(capacity=12, seed=0)
    first = _ep("a", [1.0, 1.0, 1.0], terminated=False)
    rb.add(first)
    cont = first.cut()
    cont.add_env_step(np.array([4.0], np.float32), 3, 10.0, terminated=True)
    rb.add(cont)  # a chunk of an episode already stored: concatenated
    assert rb.get_num_episodes() == 1 and len(rb) == 4
    b = rb.sample(2000, n_step=3, gamma=0.5)
    t = b["obs"][:, 0].astype(int)
    exp_r = {0: 1 + 0.5 + 0.25, 1: 1 + 0.5 + 2.5, 2: 1 + 5.0, 3: 10.0}
    for ti, r in exp_r.items():
        assert np.allclose(b["rewards"][t == ti], r)
    assert np.all(b["terminateds"][t >= 1] == 1) and np.all(b["terminateds"][t == 0] == 0)
    assert np.allclose(b["discounts"][t == 0], 0.125) and np.allclose(b["discounts"][t == 3], 0.5)
    assert np.all(b["next_obs"][:, 0][t == 0] == 3)
    for i in range(5):
        rb.add(_ep(f"x{i}", [0.0] * 4))
    assert len(rb) <= 12 and "a" not in rb.episodes


class _MyModule(TorchRLModule, ValueFunctionAPI):
    def setup(self):
        h = self.model_config.get("hidden", 64)
        d = self.observation_space.shape[0]
        self.pi = nn.Sequential(nn.Linear(d, h), nn.Tanh(), nn.Linear(h, self.action_space.n))
        self.v = nn.Sequential(nn.Linear(d, h), nn.Tanh(), nn.Linear(h, 1))

    def _forward(self, batch, **kw):
        return {Columns.ACTION_DIST_INPUTS: self.pi(batch[Columns.OBS].float())}

    def compute_values(self, batch, embeddings=None):
        return self.v(batch[Columns.OBS].float()).squeeze(-1)


_CALLS = {"loss": 0, "opt": 0}


class _MyLearner(PPOTorchLearner):
    def configure_optimizers_for_module(self, module_id, config):
        _CALLS["opt"] += 1
        self.register_optimizer(module_id=module_id,
                                optimizer=torch.optim.Adam(self.module.parameters(),
                                                           lr=config["lr"]))

    def compute_loss_for_module(self, module_id, config, batch, fwd_out):
        _CALLS["loss"] += 1
        logits = fwd_out[Columns.ACTION_DIST_INPUTS]
        lp = torch.log_softmax(logits, -1).gather(
            -1, batch[Columns.ACTIONS].long()[:, None])[:, 0]
        ratio = torch.exp(lp - batch[Columns.ACTION_LOGP])
        adv = batch[Columns.ADVANTAGES]
        surr = torch.minimum(ratio * adv, ratio.clamp(0.8, 1.2) * adv)
        vf = ((fwd_out[Columns.VF_PREDS] - batch[Columns.VALUE_TARGETS]) ** 2).mean()
        return -surr.mean() + 0.5 * vf


def test_ppo_user_module_and_custom_loss(cluster):
    cfg = (PPOConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=2, num_envs_per_env_runner=4)
           .training(train_batch_size=2000, minibatch_size=250, num_epochs=8, lr=3e-3,
                     lambda_=0.95, learner_class=_MyLearner)
           .rl_module(rl_module_spec=RLModuleSpec(module_class=_MyModule,
                                                  model_config={"hidden": 64}))
           .debugging(seed=0))
    algo = cfg.build()
    best = 0.0
    for _ in range(15):
        best = max(best, algo.train()["env_runners"]["episode_return_mean"])
        if best > 120:
            break
    assert best > 120
    assert _CALLS["opt"] == 1 and _CALLS["loss"] > 0
    m = algo.get_module()
    assert isinstance(m.m, _MyModule)  # the user's module, with the trained weights
    a = algo.compute_single_action(np.zeros(4, np.float32))
    assert a in (0, 1)
    algo.stop()


def test_lstm_ppo_solves_memory_env(cluster):
    def run(use_lstm, iters):
        cfg = (PPOConfig().environment("RepeatAfterMeEnv", env_config={"episode_len": 20})
               .env_runners(num_env_runners=2, num_envs_per_env_runner=8,
                            rollout_fragment_length=20)
               .training(train_batch_size=640, minibatch_size=160, num_epochs=6, lr=3e-3,
                         gamma=0.9, lambda_=0.95, vf_loss_coeff=0.5, kl_coeff=0.0)
               .rl_module(model_config={"use_lstm": use_lstm, "lstm_cell_size": 32,
                                        "fcnet_hiddens": [32]})
               .debugging(seed=1))
        algo = cfg.build()
        r = None
        for _ in range(iters):
            r = algo.train()["env_runners"]["episode_return_mean"]
            if use_lstm and r > 16:
                break
        state = algo.get_module().get_initial_state()
        algo.stop()
        return r, state

    r_lstm, st = run(True, 30)
    assert r_lstm > 16 and set(st) == {"h", "c"}  # near the optimum of 19
    r_ff, st_ff = run(False, 10)
    assert abs(r_ff) < 6  # a memoryless policy cannot beat chance (0)


def test_dqn_from_episode_replay_buffer(cluster):
    cfg = (DQNConfig().environment("CartPole-v1")
           .env_runners(num_env_runners=0, rollout_fragment_length=8)
           .training(replay_buffer_config={"type": "EpisodeReplayBuffer", "capacity": 50000},
                     n_step=3, lr=1e-3, train_batch_size=64, training_intensity=32,
                     num_steps_sampled_before_learning_starts=500,
                     target_network_update_freq=250, epsilon=[(0, 1.0), (5000, 0.02)])
           .rl_module(model_config={"fcnet_hiddens": [64], "fcnet_activation": "relu"})
           .debugging(seed=0))
    algo = cfg.build()
    assert type(algo.buffer).__name__ == "EpisodeReplayBuffer"
    best = 0.0  # best smoothed return after 3000 steps (a random policy averages ~22)
    for _ in range(2500):
        res = algo.train()
        if res["num_env_steps_sampled_lifetime"] > 3000:
            best = max(best, res["env_runners"]["episode_return_mean"])
        if best > 45:
            break
    assert best > 45
    assert algo.buffer.get_num_episodes() > 10
    algo.stop()


def test_single_agent_episode_setters_and_batches():
    """SingleAgentEpisode: env_steps()/agent_steps(), validate, set_* overwrites, and the
    chunk as a column dict / SampleBatch (reference: single_agent_episode.py)."""
    import numpy as np

    from ray_amd.rllib.env.single_agent_episode import SingleAgentEpisode

    e = SingleAgentEpisode()
    e.add_env_reset(np.zeros(2))
    for i in range(4):
        e.add_env_step(np.full(2, i + 1.0), i, 1.0, extra_model_outputs={"logp": -0.5},
                       terminated=i == 3)
    e.validate()
    assert e.env_steps() == e.agent_steps() == 4
    e.set_rewards(new_data=[5.0, 6.0], at_indices=slice(1, 3))
    e.set_actions(new_data=7, at_indices=0)
    e.set_extra_model_outputs(key="vf", new_data=[0.1, 0.2, 0.3, 0.4])
    assert e.get_rewards() == [1.0, 5.0, 6.0, 1.0] and e.get_actions()[0] == 7
    d = e.get_data_dict()
    assert d["obs"].shape == (4, 2) and np.array_equal(d["new_obs"][:, 0], [1, 2, 3, 4])
    assert d["terminateds"].tolist() == [False, False, False, True]
    assert d["vf"].tolist() == [0.1, 0.2, 0.3, 0.4]
    sb = e.get_sample_batch()
    assert len(sb["rewards"]) == 4
    e.finalize()
    assert e.is_finalized
    import pytest as _pt

    with _pt.raises(ValueError):
        e.set_rewards(new_data=0.0, at_indices=0)
