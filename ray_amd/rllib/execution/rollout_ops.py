"""``synchronous_parallel_sample`` (reference: rllib/execution/rollout_ops.py): one
sampling round over an algorithm's env runners (or its local runner), concatenated."""

from __future__ import annotations


def synchronous_parallel_sample(*, worker_set=None, max_agent_steps=None,
                                max_env_steps=None, concat=True, sample_timeout_s=None,
                                **kwargs):
    """``worker_set``: an Algorithm (or its ``env_runner_group``). Samples until
    ``max_env_steps`` env steps (one round when None)."""
    import ray_amd as ray

    algo = getattr(worker_set, "algo", worker_set)
    batches, steps = [], 0
    target = max_env_steps or max_agent_steps
    while True:
        if algo._runners.num_actors():
            got = ray.get([r.sample.remote() for r in algo._runners.actors()],
                          timeout=sample_timeout_s)
        else:
            got = [algo.local_runner.sample()]
        batches.extend(got)
        steps += sum(int(b.get("env_steps", 0)) for b in got)
        if target is None or steps >= target:
            break
    if not concat:
        return batches
    from ray_amd.rllib.core.learner import concat_batches

    return concat_batches(batches)
