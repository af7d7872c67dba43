"""RLlib PPO synthetic-Atari throughput bench (BASELINE.json config 3).

Config follows rllib/tuned_examples/ppo/atari-ppo.yaml (train_batch_size 5000,
rollout_fragment_length 100, minibatch 500, 10 epochs, clip 0.1, lambda 0.95,
kl_coeff 0.5, entropy 0.01, vf_share_layers) with 8 env-runner actors x 5 envs
(CPU sampling, Nature-CNN inference) and 1 MI355X learner (bf16 CNN, HIP GAE +
fused PPO loss + fused AdamW). Metric: env steps per second through complete
train() iterations (sampling + learning + weight sync).
"""

from __future__ import annotations

import json
import os
import time


def _learners(args):
    """--gpus N: N GPU learners in one RCCL group (LearnerGroup over a Train WorkerGroup,
    the gradient all-reduce on RCCL / xGMI), weak scaling: 8 env runners and one
    train-batch worth of samples per learner. N = 1 keeps the local learner."""
    n = max(1, int(getattr(args, "gpus", 1) or 1))
    return n, (n if n > 1 else 0)


def _envs_per_runner() -> int:
    """Vectorised envs per EnvRunner (RAY_AMD_RUNNER_ENVS, default 5 as in the reference's
    atari-ppo example). The runners' Nature-CNN inference runs on CPU: a bigger batch per
    forward amortises it (one runner, 1 thread, this container's CPU: 5 envs 2.5k, 20 envs
    4.5k, 40 envs 4.7k env-steps/s)."""
    return int(os.environ.get("RAY_AMD_RUNNER_ENVS", "5"))


def _inference_where(runner_gpus: float, server_gpus: float = 0.0) -> str:
    """Where the env runners' policy forward runs (reported in the JSON line)."""
    if server_gpus > 0:
        return ("gpu policy server (all runners' envs batched into one HIP graph per step, "
                "shared-memory mailbox; in the learner's process with a local learner)")
    if runner_gpus <= 0:
        return "cpu (bf16 Nature-CNN, torch)"
    if os.environ.get("RAY_AMD_RUNNER_GRAPH", "1") == "1":
        return "gpu (one HIP graph per step: conv.hip MFMA convs, Gumbel-max draw)"
    return "gpu (eager)"


def bench_ppo(args):
    import ray_amd as ray
    from ray_amd.rllib.algorithms import PPOConfig

    n_gpus, n_learners = _learners(args)
    n_runners = int(os.environ.get("RAY_AMD_PPO_RUNNERS", str(8 * n_gpus)))
    ray.init(num_cpus=max(n_runners + n_gpus + 2, os.cpu_count() or 1), num_gpus=n_gpus,
             ignore_reinit_error=True)
    # env-runner policy inference device: fractional MI355X shares (8 x 0.125) or CPU (0)
    runner_gpus = float(os.environ.get("RAY_AMD_RUNNER_GPUS", "0"))
    # > 0: one batched GPU policy server for all runners (rllib/env/policy_server.py). The
    # default with a local learner: the server is a thread of the learner's process
    # (profiles/r6/README.md r6i: 56k sync / 84-89k async against 44-47k / 54-71k with CPU
    # inference on the same boxes)
    import torch

    default_srv = "0.5" if n_learners == 0 and torch.cuda.is_available() else "0"
    server_gpus = float(os.environ.get("RAY_AMD_POLICY_SERVER_GPUS", default_srv))
    sample_async = os.environ.get("RAY_AMD_PPO_ASYNC", "0") == "1"
    # CPU threads per env runner (torch intra-op threads for the Nature-CNN inference)
    runner_cpus = float(os.environ.get("RAY_AMD_RUNNER_CPUS", "1"))
    # rollout_fragment_length "auto": 5000 / (runners x 5 envs) per env, so one sampling
    # round is exactly train_batch_size env steps (atari-ppo.yaml uses 10 x 5 x 100)
    cfg = (PPOConfig().environment("SyntheticAtari-v0")
           .env_runners(num_env_runners=n_runners, num_envs_per_env_runner=_envs_per_runner(),
                        rollout_fragment_length="auto", num_gpus_per_env_runner=runner_gpus,
                        num_cpus_per_env_runner=runner_cpus, sample_async=sample_async,
                        num_gpus_per_policy_server=server_gpus)
           .training(train_batch_size=5000 * n_gpus, minibatch_size=500, num_epochs=10,
                     lr=1e-4, lambda_=0.95, kl_coeff=0.5, clip_param=0.1, vf_clip_param=10.0,
                     entropy_coeff=0.01, model={"vf_share_layers": True})
           .learners(num_learners=n_learners, num_gpus_per_learner=1)
           .debugging(seed=0))
    algo = cfg.build()
    for _ in range(args.warmup):
        algo.train()
    t0 = time.perf_counter()
    steps = 0
    learn_stats = {}
    per_iter = []
    for _ in range(args.steps):
        r = algo.train()
        steps += r["num_env_steps_sampled_this_iter"]
        per_iter.append(r["num_env_steps_sampled_this_iter"])
        learn_stats = r["learners"]
    dt = time.perf_counter() - t0
    value = steps / dt
    print(json.dumps({
        "metric": "rllib_ppo_synthetic_atari_env_steps_per_sec",
        "value": round(value, 1), "unit": "env_steps/s", "n_gpus": n_gpus, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1000, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic",
        "config": {"model": "nature-cnn-ppo", "env": "SyntheticAtari-v0 84x84x4",
                   "env_runners": n_runners, "envs_per_runner": _envs_per_runner(),
                   "train_batch_size": 5000 * n_gpus,
                   "env_steps_per_iter_measured": sorted(set(per_iter)),
                   "rollout_fragment_length": algo.config.rollout_fragment_length,
                   "minibatch_size": 500, "num_epochs": 10,
                   "parallelism": f"{n_gpus} learner{'s' if n_gpus > 1 else ''}",
                   "env_runner_gpus": runner_gpus, "env_runner_cpus": runner_cpus,
                   "env_runner_inference": _inference_where(runner_gpus, server_gpus),
                   "sample_async": sample_async},
        "learner": {k: learn_stats.get(k) for k in ("total_loss", "entropy", "mean_kl_loss",
                                                     "sample_time_s", "sample_wait_s",
                                                     "learn_time_s", "sync_time_s")},
    }), flush=True)
    algo.stop()
    ray.shutdown()


def bench_impala(args):
    """RLlib IMPALA synthetic-Atari throughput (BASELINE.json config 5): asynchronous
    env-runner sampling + V-trace HIP kernel learners; ``--gpus N`` runs N learners on N
    MI355X joined by RCCL (the config's 8-learner form at N = 8)."""
    import ray_amd as ray
    from ray_amd.rllib.algorithms import IMPALAConfig

    n_gpus, n_learners = _learners(args)
    n_runners = int(os.environ.get("RAY_AMD_PPO_RUNNERS", str(8 * n_gpus)))
    ray.init(num_cpus=max(n_runners + n_gpus + 2, os.cpu_count() or 1), num_gpus=n_gpus,
             ignore_reinit_error=True)
    cfg = (IMPALAConfig().environment("SyntheticAtari-v0")
           .env_runners(num_env_runners=n_runners, num_envs_per_env_runner=_envs_per_runner(),
                        rollout_fragment_length=50)
           .training(train_batch_size=500 * n_gpus, lr=6e-4, vf_loss_coeff=0.5,
                     entropy_coeff=0.01, grad_clip=40.0)
           .learners(num_learners=n_learners, num_gpus_per_learner=1)
           .debugging(seed=0))
    cfg.min_time_s_per_iteration = 2.0
    algo = cfg.build()
    for _ in range(args.warmup):
        algo.train()
    t0 = time.perf_counter()
    steps = 0
    for _ in range(args.steps):
        r = algo.train()
        steps += r["num_env_steps_sampled_this_iter"]
    dt = time.perf_counter() - t0
    print(json.dumps({
        "metric": "rllib_impala_synthetic_atari_env_steps_per_sec",
        "value": round(steps / dt, 1), "unit": "env_steps/s", "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1000, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic",
        "config": {"model": "nature-cnn-impala", "env": "SyntheticAtari-v0 84x84x4",
                   "env_runners": n_runners, "envs_per_runner": _envs_per_runner(), "rollout_fragment_length": 50,
                   "train_batch_size": 500 * n_gpus,
                   "parallelism": f"{n_gpus} learner{'s' if n_gpus > 1 else ''}"},
    }), flush=True)
    algo.stop()
    ray.shutdown()
