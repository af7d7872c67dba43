"""Programmatic autoscaler requests (reference: python/ray/autoscaler/sdk/sdk.py
request_resources)."""

from __future__ import annotations

import pickle


def request_resources(num_cpus: int | None = None, bundles: list | None = None) -> None:
    """Ask the autoscaler to scale to fit `num_cpus` CPUs and/or `bundles` immediately,
    regardless of task demand. A later call replaces the request; ``request_resources()``
    with no arguments clears it."""
    from ray_amd._private import worker as W

    req = []
    if num_cpus:
        req.extend({"CPU": 1.0} for _ in range(int(num_cpus)))
    for b in bundles or []:
        req.append({k: float(v) for k, v in b.items()})
    W.global_worker.core.call_raylet("kv_put", "__autoscaler", b"resource_request",
                                     pickle.dumps(req), True)
