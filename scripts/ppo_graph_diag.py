#!/usr/bin/env python
"""Bisect the PPO learner HIP-graph step: gradient norm seen by each optimizer step."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_amd.rllib.algorithms import PPOConfig  # noqa: E402
from ray_amd.rllib.core.learner import Learner  # noqa: E402
from ray_amd.rllib.env import make_env  # noqa: E402

cfg = (PPOConfig().environment("SyntheticAtari-v0")
       .training(train_batch_size=1000, minibatch_size=500, num_epochs=2, lr=3e-4,
                 model={"vf_share_layers": True})).to_dict()
env = make_env("SyntheticAtari-v0")
lr = Learner(cfg, env.observation_space, env.action_space)
T, B = 20, 50
rng = np.random.default_rng(0)
obs = rng.integers(0, 256, (T, B, 84, 84, 4), dtype=np.uint8)
acts = rng.integers(0, env.action_space.n, (T, B))
batch = {"obs": obs, "rewards": np.where(acts == 0, 1.0, -1.0).astype(np.float32),
         "terminateds": np.ones((T, B), np.float32), "actions": acts,
         "action_logp": np.full((T, B), -np.log(env.action_space.n), np.float32),
         "action_dist_inputs": np.zeros((T, B, env.action_space.n), np.float32),
         "bootstrap_obs": rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)}
orig_step = lr.opt.step
orig_replay = torch.cuda.CUDAGraph.replay


def replay(self):
    torch.cuda.synchronize()
    print(f"    before replay g {lr.flat.g.float().norm().item():.4e} idx "
          f"{lr._graph_io[0][:4].tolist()}", flush=True)
    orig_replay(self)
    torch.cuda.synchronize()
    print(f"    after replay g {lr.flat.g.float().norm().item():.4e} stats "
          f"{lr._graph_io[1].tolist()}", flush=True)


def step(*a, **k):
    torch.cuda.synchronize()
    print(f"    opt.step sees g {lr.flat.g.float().norm().item():.4e}", flush=True)
    return orig_step(*a, **k)


torch.cuda.CUDAGraph.replay = replay
lr.opt.step = step
for i in range(2):
    print(f"update {i}", flush=True)
    st = lr.update_ppo(batch)
    print(f"  kl {st['mean_kl_loss']:.3e} m {lr.opt.m.norm().item():.3e}", flush=True)
