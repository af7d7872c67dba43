#!/usr/bin/env python
"""Env-runner policy inference cost on the host CPU: Nature-CNN, 5 frames per step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from ray_amd.rllib.core.rl_module import RLModule  # noqa: E402
from ray_amd.rllib.env import make_env  # noqa: E402

env = make_env("SyntheticAtari-v0")
x = torch.randint(0, 256, (5, 84, 84, 4), dtype=torch.uint8)
for threads in (1, 2):
    torch.set_num_threads(threads)
    for dtype in (torch.float32, torch.bfloat16):
        for cl in (False, True):
            m = RLModule(env.observation_space, env.action_space, {"vf_share_layers": True})
            m.eval()
            if cl:
                m = m.to(memory_format=torch.channels_last)
            with torch.no_grad():
                def f():
                    if dtype == torch.bfloat16:
                        with torch.autocast("cpu", dtype=torch.bfloat16):
                            return m.forward_inference(x)
                    return m.forward_inference(x)
                for _ in range(5):
                    f()
                t0 = time.perf_counter()
                for _ in range(50):
                    f()
                dt = (time.perf_counter() - t0) / 50
            print(f"threads={threads} {dtype} channels_last={cl}: {dt * 1e3:.3f} ms/step", flush=True)
