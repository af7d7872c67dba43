#!/usr/bin/env python
"""Capture variants of the PPO learner body in a HIP graph; compare replayed flat grads
with an eager run of the same body (same idx)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_amd.ops import functional as rf  # noqa: E402
from ray_amd.rllib.algorithms import PPOConfig  # noqa: E402
from ray_amd.rllib.core.learner import Learner  # noqa: E402
from ray_amd.rllib.env import make_env  # noqa: E402

cfg = (PPOConfig().environment("SyntheticAtari-v0")
       .training(train_batch_size=1000, minibatch_size=500, num_epochs=2, lr=3e-4,
                 model={"vf_share_layers": True})).to_dict()
env = make_env("SyntheticAtari-v0")
L = Learner(cfg, env.observation_space, env.action_space)
dev = torch.device("cuda")
N, A = 1000, env.action_space.n
obs = torch.randint(0, 256, (N, 84, 84, 4), dtype=torch.uint8, device=dev)
aux = rf.ppo_pack(torch.zeros(N, A, device=dev), torch.randint(0, A, (N,), device=dev),
                  torch.full((N,), -float(np.log(A)), device=dev), torch.randn(N, device=dev),
                  torch.randn(N, device=dev))
idx = torch.randperm(N, device=dev)[:500]
params = L.flat.params()
grads = [p._ra_grad for p in params]
one = torch.ones((), device=dev)
stats = torch.zeros(6, device=dev)
kl_dev = torch.full((1,), 0.2, device=dev)


def body(variant):
    L.flat.g.zero_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out = L.module.forward_train(obs, idx=idx)
    loss = rf.ppo_loss_packed(out["action_dist_inputs"], out["vf_preds"], aux, idx, stats,
                              clip=0.3, kl_coeff=0.2, kl_dev=kl_dev)
    if variant == "backward":
        loss.backward(one)
        return
    gs = torch.autograd.grad(loss, params, grad_outputs=one, allow_unused=True)
    dst = [g for g, x in zip(grads, gs) if x is not None]
    src = [x for x in gs if x is not None]
    if variant == "foreach":
        torch._foreach_copy_(dst, src)
    else:
        for d, s in zip(dst, src):
            d.copy_(s)


for variant in ("foreach", "loop", "backward"):
    body(variant)
    torch.cuda.synchronize()
    ref = L.flat.g.float().clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            body(variant)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body(variant)
    torch.cuda.synchronize()
    after_cap = L.flat.g.float().norm().item()
    L.flat.g.fill_(7.0)
    g.replay()
    torch.cuda.synchronize()
    got = L.flat.g.float()
    per = {n: round((got[o:o + p.numel()] - ref[o:o + p.numel()]).norm().item(), 5)
           for (n, p), o in zip(L.flat.order, L.flat.offsets)}
    print(f"{variant}: ref {ref.norm().item():.4e} after-capture {after_cap:.4e} replay "
          f"{got.norm().item():.4e} diff {(got - ref).norm().item():.4e}", flush=True)
    print("   per-param diff", per, flush=True)
