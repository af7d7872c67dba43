#!/usr/bin/env python
"""GPU sanity check: does the PPO learner (HIP graph + fused conv path) actually learn?
Synthetic Atari batch where action 0 has advantage +1 and others -1 (via rewards);
prints encoder activation scale vs a CPU fp32 copy, and per-update KL / entropy."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from ray_amd.rllib.algorithms import PPOConfig  # noqa: E402
from ray_amd.rllib.core.learner import Learner  # noqa: E402
from ray_amd.rllib.core.rl_module import RLModule  # noqa: E402
from ray_amd.rllib.env import make_env  # noqa: E402


def run(graph):
    cfg = (PPOConfig().environment("SyntheticAtari-v0")
           .training(train_batch_size=2000, minibatch_size=500, num_epochs=4, lr=3e-4,
                     model={"vf_share_layers": True})).to_dict()
    cfg["learner_cuda_graph"] = graph
    env = make_env("SyntheticAtari-v0")
    lr = Learner(cfg, env.observation_space, env.action_space)
    T, B = 40, 50
    rng = np.random.default_rng(0)
    obs = rng.integers(0, 256, (T, B, 84, 84, 4), dtype=np.uint8)
    acts = rng.integers(0, env.action_space.n, (T, B))
    batch = {"obs": obs, "rewards": np.where(acts == 0, 1.0, -1.0).astype(np.float32),
             "terminateds": np.ones((T, B), np.float32),
             "actions": acts,
             "action_logp": np.full((T, B), -np.log(env.action_space.n), np.float32),
             "action_dist_inputs": np.zeros((T, B, env.action_space.n), np.float32),
             "bootstrap_obs": rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)}
    x = torch.from_numpy(obs[0, :8]).cuda()
    with torch.no_grad():
        h_gpu = lr.module.encoder(x).float().cpu()
        cpu = RLModule(env.observation_space, env.action_space, cfg.get("model"))
        cpu.load_state_dict({k: v.float().cpu() for k, v in lr.module.state_dict().items()})
        h_cpu = cpu.encoder(torch.from_numpy(obs[0, :8]))
    print(f"graph={graph} encoder |h| gpu {h_gpu.abs().mean():.4f} cpu {h_cpu.abs().mean():.4f} "
          f"rel {((h_gpu - h_cpu).norm() / h_cpu.norm()).item():.4f}", flush=True)
    for i in range(4):
        p0 = lr.flat.p32.clone()
        st = lr.update_ppo(batch)
        print(f"  dp32 {(lr.flat.p32 - p0).norm().item():.3e} last_norm "
              f"{lr.opt.last_norm.item():.3e} m {lr.opt.m.norm().item():.3e} "
              f"v {lr.opt.v.norm().item():.3e} step {lr.opt.step_count} "
              f"g {lr.flat.g.float().norm().item():.3e} clip {lr.opt.max_grad_norm}", flush=True)
        with torch.no_grad():
            p = torch.softmax(lr.module.forward_train(torch.from_numpy(obs[0]).cuda())[
                "action_dist_inputs"].float(), -1)[:, 0].mean().item()
        print(f"  update {i}: kl {st['mean_kl_loss']:.3e} entropy {st['entropy']:.5f} "
              f"policy_loss {st['policy_loss']:.4f} p(a=0) {p:.4f}", flush=True)


if __name__ == "__main__" and not os.environ.get("DIAG"):
    run(True)
    run(False)


def diag():
    """Replay the captured SGD step once and report which gradient views were written."""
    cfg = (PPOConfig().environment("SyntheticAtari-v0")
           .training(train_batch_size=2000, minibatch_size=500, num_epochs=1, lr=3e-4,
                     model={"vf_share_layers": True})).to_dict()
    env = make_env("SyntheticAtari-v0")
    lr = Learner(cfg, env.observation_space, env.action_space)
    T, B = 40, 50
    rng = np.random.default_rng(0)
    obs = rng.integers(0, 256, (T, B, 84, 84, 4), dtype=np.uint8)
    acts = rng.integers(0, env.action_space.n, (T, B))
    batch = {"obs": obs, "rewards": np.where(acts == 0, 1.0, -1.0).astype(np.float32),
             "terminateds": np.ones((T, B), np.float32), "actions": acts,
             "action_logp": np.full((T, B), -np.log(env.action_space.n), np.float32),
             "action_dist_inputs": np.zeros((T, B, env.action_space.n), np.float32),
             "bootstrap_obs": rng.integers(0, 256, (B, 84, 84, 4), dtype=np.uint8)}
    lr.update_ppo(batch)
    idx_buf, _ = lr._graph_io
    idx_buf.copy_(torch.arange(500, device="cuda"))
    lr._graph.replay()
    torch.cuda.synchronize()
    for n, p in lr.flat.order:
        print(f"  graph grad {n:28s} {p._ra_grad.float().norm().item():.4e}", flush=True)
    # the same body eagerly
    lr.flat.g.zero_()
    out = lr.module.forward_train(lr._graph_bufs[0], idx=idx_buf)
    from ray_amd.ops import functional as rf
    stats = torch.zeros(6, device="cuda")
    loss = rf.ppo_loss_packed(out["action_dist_inputs"], out["vf_preds"], lr._graph_bufs[1],
                              idx_buf, stats, clip=0.3, kl_coeff=0.2)
    gs = torch.autograd.grad(loss, lr.flat.params(), grad_outputs=torch.ones((), device="cuda"),
                             allow_unused=True)
    for (n, p), g in zip(lr.flat.order, gs):
        gn = g.float().norm().item() if g is not None else None
        print(f"  eager {n:28s} sink {p._ra_grad.float().norm().item():.4e} ret {gn}", flush=True)


if __name__ == "__main__" and os.environ.get("DIAG"):
    diag()
