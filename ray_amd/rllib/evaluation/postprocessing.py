"""Advantage postprocessing (reference: rllib/evaluation/postprocessing.py). The learners
of this framework compute GAE with the HIP kernel (``ops.functional.gae``); these are the
numpy forms for user code and old-stack policies."""

from __future__ import annotations

import numpy as np


class Postprocessing:
    ADVANTAGES = "advantages"
    VALUE_TARGETS = "value_targets"


def discount_cumsum(x: np.ndarray, gamma: float) -> np.ndarray:
    """``y[t] = sum_k gamma^k x[t+k]`` over the (last) time axis."""
    x = np.asarray(x, dtype=np.float64)
    out = np.zeros_like(x)
    run = 0.0
    for t in range(len(x) - 1, -1, -1):
        run = x[t] + gamma * run
        out[t] = run
    return out.astype(np.float32)


def compute_advantages(rollout, last_r: float, gamma: float = 0.9, lambda_: float = 1.0,
                       use_gae: bool = True, use_critic: bool = True, rewards=None,
                       vf_preds=None):
    """Adds ``advantages`` and ``value_targets`` to ``rollout`` (a dict / SampleBatch of
    one trajectory with ``rewards`` and, for GAE, ``vf_preds``)."""
    r = np.asarray(rewards if rewards is not None else rollout["rewards"], np.float64)
    v = np.asarray(vf_preds if vf_preds is not None else rollout.get("vf_preds", np.zeros_like(r)),
                   np.float64)
    if use_gae:
        if not use_critic:
            raise ValueError("use_gae=True needs use_critic=True")
        vpred_t = np.concatenate([v, [last_r]])
        delta = r + gamma * vpred_t[1:] - vpred_t[:-1]
        adv = discount_cumsum(delta, gamma * lambda_)
        targets = (adv + v).astype(np.float32)
    else:
        rt = np.concatenate([r, [last_r]])
        disc = discount_cumsum(rt, gamma)[:-1]
        adv = (disc - v).astype(np.float32) if use_critic else disc
        targets = disc.astype(np.float32) if use_critic else np.zeros_like(disc)
    rollout[Postprocessing.ADVANTAGES] = np.asarray(adv, np.float32)
    rollout[Postprocessing.VALUE_TARGETS] = np.asarray(targets, np.float32)
    return rollout


def compute_gae_for_sample_batch(policy, sample_batch, other_agent_batches=None,
                                 episode=None):
    """GAE over one trajectory batch, bootstrapping from ``policy``'s value of the last
    next observation unless the trajectory terminated."""
    cfg = getattr(policy, "config", {}) or {}
    terms = sample_batch.get("terminateds", sample_batch.get("dones"))
    last_r = 0.0
    if terms is not None and len(terms) and not bool(np.asarray(terms)[-1]):
        vf = getattr(policy, "compute_value", None) or getattr(policy, "value", None)
        if vf is not None:
            last_r = float(np.asarray(vf(np.asarray(sample_batch["new_obs"])[-1:]))[0])
    return compute_advantages(sample_batch, last_r, cfg.get("gamma", 0.99),
                              cfg.get("lambda", 1.0), cfg.get("use_gae", True),
                              cfg.get("use_critic", True))
