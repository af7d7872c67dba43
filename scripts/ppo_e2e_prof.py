#!/usr/bin/env python
"""cProfile two synchronous PPO iterations of the bench config (where does the driver's
wall time go besides sample / learn / sync?)."""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import ray_amd as ray  # noqa: E402
from ray_amd.rllib.algorithms import PPOConfig  # noqa: E402

ray.init(num_cpus=10)
cfg = (PPOConfig().environment("SyntheticAtari-v0")
       .env_runners(num_env_runners=8, num_envs_per_env_runner=5, rollout_fragment_length="auto")
       .training(train_batch_size=5000, minibatch_size=500, num_epochs=10, lr=1e-4,
                 lambda_=0.95, kl_coeff=0.5, clip_param=0.1, vf_clip_param=10.0,
                 entropy_coeff=0.01, model={"vf_share_layers": True})
       .learners(num_learners=0, num_gpus_per_learner=1).debugging(seed=0))
algo = cfg.build()
for _ in range(2):
    algo.train()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(3):
    r = algo.train()
    print({k: round(v, 4) for k, v in r["learners"].items() if k.endswith("_s")},
          round(r["time_this_iter_s"], 4), flush=True)
pr.disable()
print("wall per iter", (time.perf_counter() - t0) / 3, flush=True)
pstats.Stats(pr).sort_stats("cumulative").print_stats(35)
algo.stop()
ray.shutdown()
