#!/usr/bin/env python
"""PPO learner-only throughput on one MI355X (the GPU half of BASELINE.json config 3):
Nature-CNN actor-critic, 5000-frame train batch of synthetic 84x84x4 uint8 frames,
10 epochs x 10 minibatches of 500, HIP GAE + fused PPO loss + flat AdamW.

    python scripts/ppo_learner_bench.py [--iters 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_amd.rllib.algorithms import PPOConfig  # noqa: E402
from ray_amd.rllib.core.learner import Learner  # noqa: E402
from ray_amd.rllib.env import make_env  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    cfg = (PPOConfig().environment("SyntheticAtari-v0")
           .training(train_batch_size=5000, minibatch_size=500, num_epochs=10, lr=1e-4,
                     model={"vf_share_layers": True})).to_dict()
    env = make_env("SyntheticAtari-v0")
    lr = Learner(cfg, env.observation_space, env.action_space)
    T, B = 100, 50
    rng = np.random.default_rng(0)
    batch = {"obs": rng.integers(0, 256, (T, B, 84, 84, 4), dtype=np.uint8),
             "rewards": rng.random((T, B), dtype=np.float32),
             "terminateds": (rng.random((T, B)) < 0.01).astype(np.float32),
             "actions": rng.integers(0, env.action_space.n, (T, B)),
             "action_logp": np.full((T, B), -np.log(env.action_space.n), np.float32),
             "action_dist_inputs": np.zeros((T, B, env.action_space.n), np.float32),
             "bootstrap_obs": rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)}
    for _ in range(a.warmup):
        lr.update_ppo(batch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        st = lr.update_ppo(batch)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.iters
    # phase: host -> HBM staging of the 141 MB frame batch alone
    t1 = time.perf_counter()
    for _ in range(a.iters):
        lr._h2d(batch["obs"], "obs")
    torch.cuda.synchronize()
    h2d = (time.perf_counter() - t1) / a.iters
    print(json.dumps({"metric": "ppo_learner_frames_per_sec", "value": round(T * B / dt, 1),
                      "ms_per_update": round(dt * 1e3, 2), "sgd_steps": st["num_minibatches"],
                      "ms_per_sgd_step": round(dt * 1e3 / st["num_minibatches"], 3),
                      "ms_obs_h2d": round(h2d * 1e3, 2),
                      "graph_captures": getattr(lr, "_n_captures", None)}), flush=True)


if __name__ == "__main__":
    main()
