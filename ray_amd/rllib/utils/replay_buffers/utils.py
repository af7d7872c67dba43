"""Replay-buffer helpers (reference: python/ray/rllib/utils/replay_buffers/utils.py)."""

from __future__ import annotations

import numpy as np


def update_priorities_in_replay_buffer(replay_buffer, config, train_batch, train_results):
    """Feed the learner's TD errors back as priorities (prioritized buffers only)."""
    if not hasattr(replay_buffer, "update_priorities"):
        return
    eps = float((config or {}).get("replay_buffer_config", {}).get(
        "prioritized_replay_eps", 1e-6)) if isinstance(config, dict) else 1e-6
    if hasattr(replay_buffer, "replay_buffers"):  # multi-agent: {pid: (idx, td)}
        prio = {}
        for pid, res in train_results.items():
            td = res.get("td_error") if isinstance(res, dict) else None
            b = train_batch[pid] if isinstance(train_batch, dict) else None
            if td is not None and b is not None and "batch_indexes" in b:
                prio[pid] = (np.asarray(b["batch_indexes"]), np.abs(np.asarray(td)) + eps)
        if prio:
            replay_buffer.update_priorities(prio)
    else:
        td = train_results.get("td_error")
        if td is not None and "batch_indexes" in train_batch:
            replay_buffer.update_priorities(np.asarray(train_batch["batch_indexes"]),
                                            np.abs(np.asarray(td)) + eps)


def sample_min_n_steps_from_buffer(replay_buffer, min_steps: int, count_by_agent_steps=False):
    """Sample batches until at least ``min_steps`` items were drawn; concatenated."""
    parts, n = [], 0
    while n < min_steps:
        b = replay_buffer.sample(min_steps - n)
        if not b:
            break
        k = len(next(iter(b.values())))
        if k == 0:
            break
        parts.append(b)
        n += k
    if not parts:
        return None
    keys = set.intersection(*[set(p) for p in parts])
    return {k: np.concatenate([np.asarray(p[k]) for p in parts]) for k in keys}


def validate_buffer_config(config) -> None:
    rb = (config or {}).get("replay_buffer_config") if isinstance(config, dict) else None
    if rb is not None and not isinstance(rb, dict):
        raise ValueError("replay_buffer_config must be a dict")
