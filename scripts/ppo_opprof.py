"""torch.profiler op table of one eager PPO SGD step (learner graph disabled) on the GPU:
which framework ops launch the learner's small kernels."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from ray_amd.rllib.algorithms import PPOConfig  # noqa: E402
from ray_amd.rllib.core.learner import Learner  # noqa: E402
from ray_amd.rllib.env import make_env  # noqa: E402

cfg = (PPOConfig().environment("SyntheticAtari-v0")
       .training(train_batch_size=5000, minibatch_size=500, num_epochs=1, lr=1e-4,
                 model={"vf_share_layers": True})).to_dict()
cfg["learner_cuda_graph"] = False
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
lr.update_ppo(batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    lr.update_ppo(batch)
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="count", row_limit=45, max_name_column_width=60))
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
             with_stack=True) as prof2:
    lr.update_ppo(batch)
    torch.cuda.synchronize()
ka = prof2.key_averages(group_by_input_shape=True, group_by_stack_n=6)
rows = [e for e in ka if e.key in ("aten::copy_", "aten::clone", "aten::_to_copy",
                                   "aten::contiguous", "aten::add_", "aten::sum")]
rows.sort(key=lambda e: -e.device_time_total)
for e in rows[:25]:
    print(f"{e.key:18s} n={e.count:4d} dev_us={e.device_time_total:9.1f} shapes={e.input_shapes}")
    for fr in (e.stack or [])[:6]:
        print("      ", fr)
