"""``rllib`` CLI (reference: rllib/scripts.py, rllib/train.py, rllib/evaluate.py).

    python -m ray_amd.rllib train --algo PPO --env CartPole-v1 \\
        --config '{"lr": 3e-4}' --stop '{"env_runners/episode_return_mean": 150}'
    python -m ray_amd.rllib train file tuned_example.yaml     # {name: {run, env, stop, config}}
    python -m ray_amd.rllib evaluate <checkpoint_dir> --algo PPO --episodes 10

``train`` runs the algorithm as a Tune experiment (``tune.run_experiments``), so stop
criteria, ``--num-samples``, grid searches in the config and checkpoint options behave as
in Tune. Tuned-example files may use old-stack keys (``num_workers``, ``num_sgd_iter``,
``sgd_minibatch_size``, ``sampler_results/episode_reward_mean``, ``timesteps_total``);
``evaluate`` restores the checkpoint and rolls out greedy (or ``--explore``) episodes on
the driver, printing one JSON summary line."""

from __future__ import annotations

import argparse
import json
import os
import sys


def _init_ray(a):
    import ray_amd as ray

    if ray.is_initialized():
        return ray
    if a.ray_address:
        ray.init(address=a.ray_address)
    else:
        kw = {}
        if a.ray_num_cpus is not None:
            kw["num_cpus"] = a.ray_num_cpus
        if a.ray_num_gpus is not None:
            kw["num_gpus"] = a.ray_num_gpus
        ray.init(**kw)
    return ray


def _load_experiments(path: str) -> dict:
    import yaml

    with open(path) as f:
        if path.endswith(".json"):
            exps = json.load(f)
        else:
            exps = yaml.safe_load(f)
    if not isinstance(exps, dict) or not exps:
        raise SystemExit(f"{path}: expected a mapping of experiment name -> spec")
    return exps


def _run(exps: dict, a) -> int:
    from ray_amd import tune

    _init_ray(a)
    specs = {}
    for name, spec in exps.items():
        spec = dict(spec)
        algo = spec.pop("run", None) or spec.pop("algo", None)
        if algo is None:
            raise SystemExit(f"experiment {name!r} names no algorithm ('run:')")
        config = dict(spec.pop("config", {}) or {})
        if spec.get("env") is not None:
            config["env"] = spec.pop("env")
        if a.framework:
            config["framework"] = a.framework
        stop = spec.pop("stop", {}) or {}
        if a.stop:
            stop = json.loads(a.stop)
        specs[name] = {
            "run": algo, "config": config, "stop": stop,
            "num_samples": spec.pop("num_samples", a.num_samples),
            "storage_path": spec.pop("storage_path", a.storage_path),
            "checkpoint_config": {
                "checkpoint_frequency": spec.pop("checkpoint_freq", a.checkpoint_freq),
                "checkpoint_at_end": spec.pop("checkpoint_at_end", a.checkpoint_at_end),
                "num_to_keep": spec.pop("keep_checkpoints_num", a.keep_checkpoints_num)},
        }
    results = []
    for name, s in specs.items():
        cc = s["checkpoint_config"]
        ana = tune.run(s["run"], config=s["config"], stop=s["stop"], name=name,
                       num_samples=s["num_samples"], storage_path=s["storage_path"],
                       checkpoint_freq=cc["checkpoint_frequency"] or 0,
                       checkpoint_at_end=cc["checkpoint_at_end"],
                       keep_checkpoints_num=cc["num_to_keep"], verbose=1)
        for t in ana.trials:
            m = t.metrics or {}
            er = m.get("env_runners") or {}
            results.append({"experiment": name, "error": repr(t.error) if t.error else None,
                            "training_iteration": m.get("training_iteration"),
                            "timesteps_total": m.get("timesteps_total"),
                            "episode_return_mean": er.get("episode_return_mean"),
                            "checkpoint": t.checkpoint.path if t.checkpoint else None})
    for r in results:
        print(json.dumps(r), flush=True)
    return 1 if any(r["error"] for r in results) else 0


def cmd_train(a) -> int:
    if a.algo is None or a.env is None:
        raise SystemExit("train needs --algo and --env (or: train file <yaml>)")
    config = json.loads(a.config) if a.config else {}
    exps = {a.experiment_name or "default": {"run": a.algo, "env": a.env, "config": config,
                                             "stop": json.loads(a.stop) if a.stop else {}}}
    a.stop = None  # already applied
    return _run(exps, a)


def cmd_train_file(a) -> int:
    return _run(_load_experiments(a.config_file), a)


def cmd_evaluate(a) -> int:
    import numpy as np

    from ray_amd.rllib.algorithms.registry import get_algorithm_class
    from ray_amd.rllib.env.envs import make_env

    _init_ray(a)
    path = a.checkpoint
    if os.path.isdir(path) and not os.path.exists(os.path.join(path, "algorithm_state.pkl")):
        cands = sorted(d for d in os.listdir(path) if d.startswith("checkpoint_"))
        if cands:  # a trial directory: its newest checkpoint
            path = os.path.join(path, cands[-1])
    algo = get_algorithm_class(a.algo).from_checkpoint(path)
    env_name = a.env or algo.config.env
    env = make_env(env_name, algo.config.env_config)
    returns, lengths, steps = [], [], 0
    while len(returns) < a.episodes and (not a.steps or steps < a.steps):
        obs, _ = env.reset(seed=None if a.seed is None else a.seed + len(returns))
        done, ret, n = False, 0.0, 0
        while not done:
            act = algo.compute_single_action(obs, explore=a.explore)
            obs, r, term, trunc, _ = env.step(act)
            ret += float(r)
            n += 1
            steps += 1
            done = term or trunc or (a.steps and steps >= a.steps)
        returns.append(ret)
        lengths.append(n)
    env.close()
    algo.stop()
    print(json.dumps({"checkpoint": path, "env": env_name, "episodes": len(returns),
                      "episode_return_mean": float(np.mean(returns)) if returns else None,
                      "episode_len_mean": float(np.mean(lengths)) if lengths else None,
                      "episode_returns": returns}), flush=True)
    return 0


def _common(p):
    p.add_argument("--ray-address", default=None)
    p.add_argument("--ray-num-cpus", type=int, default=None)
    p.add_argument("--ray-num-gpus", type=int, default=None)
    p.add_argument("--framework", default=None, choices=[None, "torch"])


def _train_opts(p):
    p.add_argument("--stop", default=None, help="JSON dict of stop criteria")
    p.add_argument("--num-samples", type=int, default=1)
    p.add_argument("--checkpoint-freq", type=int, default=0)
    p.add_argument("--checkpoint-at-end", action="store_true")
    p.add_argument("--keep-checkpoints-num", type=int, default=None)
    p.add_argument("--storage-path", default=None)
    _common(p)


def build_parser():
    ap = argparse.ArgumentParser(prog="rllib", description="ray_amd RLlib CLI")
    sub = ap.add_subparsers(dest="cmd", required=True)
    t = sub.add_parser("train", help="train an algorithm (or: train file <yaml>)")
    tsub = t.add_subparsers(dest="train_cmd")
    f = tsub.add_parser("file", help="run the experiments of a tuned-example YAML/JSON file")
    f.add_argument("config_file")
    _train_opts(f)
    f.set_defaults(fn=cmd_train_file)
    t.add_argument("--algo", "--run", dest="algo", default=None)
    t.add_argument("--env", default=None)
    t.add_argument("--config", default=None, help="JSON dict of algorithm config")
    t.add_argument("--experiment-name", default=None)
    _train_opts(t)
    t.set_defaults(fn=cmd_train)
    e = sub.add_parser("evaluate", help="roll out a checkpointed policy")
    e.add_argument("checkpoint")
    e.add_argument("--algo", "--run", dest="algo", required=True)
    e.add_argument("--env", default=None)
    e.add_argument("--episodes", type=int, default=10)
    e.add_argument("--steps", type=int, default=0)
    e.add_argument("--explore", action="store_true")
    e.add_argument("--seed", type=int, default=None)
    _common(e)
    e.set_defaults(fn=cmd_evaluate)
    return ap


def main(argv=None) -> int:
    a = build_parser().parse_args(argv)
    return a.fn(a)


if __name__ == "__main__":
    sys.exit(main())
