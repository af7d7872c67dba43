"""``collect_metrics`` / ``summarize_episodes`` (reference: python/ray/rllib/evaluation/
metrics.py): episode statistics gathered from env runners."""

from __future__ import annotations

from typing import List

import numpy as np


def summarize_episodes(episode_returns: List[float], episode_lengths: List[int],
                       custom_metrics=None) -> dict:
    r = np.asarray(episode_returns, np.float64)
    ln = np.asarray(episode_lengths, np.float64)
    nan = float("nan")
    return {"episode_reward_max": float(r.max()) if len(r) else nan,
            "episode_reward_min": float(r.min()) if len(r) else nan,
            "episode_reward_mean": float(r.mean()) if len(r) else nan,
            "episode_len_mean": float(ln.mean()) if len(ln) else nan,
            "episodes_this_iter": int(len(r)), "hist_stats": {
                "episode_reward": r.tolist(), "episode_lengths": ln.tolist()},
            "custom_metrics": dict(custom_metrics or {})}


def collect_episodes(workers=None, remote_worker_ids=None, timeout_seconds: int = 180):
    """(returns, lengths) drained from every env runner of ``workers`` (an Algorithm's
    env_runner_group, or a list of runners / actor handles)."""
    import ray_amd as ray

    runners = workers
    if hasattr(workers, "foreach_env_runner"):
        mets = workers.foreach_env_runner(lambda w: w.get_metrics())
    else:
        mets = []
        for w in runners or []:
            m = w.get_metrics.remote() if hasattr(w, "get_metrics") and \
                hasattr(w.get_metrics, "remote") else w.get_metrics()
            mets.append(m)
        mets = [ray.get(m) if isinstance(m, ray.ObjectRef) else m for m in mets]
    rets, lens = [], []
    for m in mets:
        rets.extend(m.get("episode_returns", []))
        lens.extend(m.get("episode_lengths", []))
    return rets, lens


def collect_metrics(workers=None, remote_worker_ids=None, to_be_collected=None,
                    keep_custom_metrics: bool = False, timeout_seconds: int = 180) -> dict:
    rets, lens = collect_episodes(workers, remote_worker_ids, timeout_seconds)
    return summarize_episodes(rets, lens)
