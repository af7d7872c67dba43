"""StandardAutoscaler: demand-driven scale up, idle-driven scale down.

Reference behaviour (python/ray/autoscaler/_private/autoscaler.py StandardAutoscaler,
resource_demand_scheduler.py get_nodes_to_launch, load_metrics.py): every update reads
the cluster load (task/actor resource shapes waiting for a node, pending placement-group
bundles, ``request_resources`` asks), bin-packs it onto the free capacity of running
and already-launching nodes, launches the cheapest node types that fit what is left
(bounded by per-type and global ``max_workers`` and ``upscaling_speed``), keeps every
type at ``min_workers`` and terminates worker nodes idle for ``idle_timeout_s``.

Design: the packing is a first-fit-decreasing over resource dicts (the reference's
utilization scorer reduces to "smallest node type that fits" for the single-resource
shapes GPU clusters use); the raylet computes idleness (no leases, all resources free)
in ``rpc_resource_load`` so no extra heartbeat exists.
"""

from __future__ import annotations

import pickle
import sys
import threading
import time
from dataclasses import dataclass, field

from ray_amd.autoscaler.node_provider import TAG_NODE_KIND, TAG_USER_NODE_TYPE


@dataclass
class NodeTypeConfig:
    resources: dict
    min_workers: int = 0
    max_workers: int = 10
    node_config: dict = field(default_factory=dict)


@dataclass
class AutoscalerConfig:
    node_types: dict  # name -> NodeTypeConfig
    max_workers: int = 20
    idle_timeout_s: float = 300.0
    upscaling_speed: float = 1.0
    update_interval_s: float = 1.0


def _fits(avail: dict, req: dict) -> bool:
    return all(avail.get(k, 0.0) + 1e-9 >= v for k, v in req.items() if v)


def _take(avail: dict, req: dict):
    for k, v in req.items():
        avail[k] = avail.get(k, 0.0) - v


def _size(req: dict) -> float:
    return sum(v * (1000.0 if k == "GPU" else 1.0) for k, v in req.items())


def pack(requests: list, bins: list) -> list:
    """First-fit-decreasing of `requests` into `bins` (mutated); returns the misfits."""
    left = []
    for r in sorted(requests, key=_size, reverse=True):
        for b in bins:
            if _fits(b, r):
                _take(b, r)
                break
        else:
            left.append(r)
    return left


class StandardAutoscaler:
    def __init__(self, config: AutoscalerConfig, provider, load_fn=None):
        self.config = config
        self.provider = provider
        self._load_fn = load_fn
        self.launched_at: dict = {}  # provider node id -> launch time
        self.events: list = []  # (time, "launch"/"terminate", node type, provider id)

    # ------------------------------------------------------------------ inputs
    def _load(self) -> dict:
        if self._load_fn is not None:
            return self._load_fn()
        from ray_amd._private import worker as W

        return W.global_worker.core.call_raylet("resource_load", timeout=30)

    def _worker_nodes(self):
        out = {}
        for nid in self.provider.non_terminated_nodes({TAG_NODE_KIND: "worker"}):
            out[nid] = self.provider.node_tags(nid).get(TAG_USER_NODE_TYPE)
        return out

    # ------------------------------------------------------------------ one round
    def update(self) -> dict:
        cfg = self.config
        load = self._load()
        demand = [dict(d) for d in load["demand"]]
        for bundles in load["pg_demand"]:
            demand.extend(dict(b) for b in bundles)
        requested = pickle.loads(load["requested"]) if load.get("requested") else []
        workers = self._worker_nodes()
        joined = {n["node_id"]: n for n in load["nodes"]}
        launching = [(pid, t) for pid, t in workers.items()
                     if self.provider.ray_node_id(pid) not in joined]
        # 1) what existing + launching capacity cannot absorb
        free = [dict(n["available"]) for n in load["nodes"]]
        free += [dict(cfg.node_types[t].resources) for _, t in launching if t in cfg.node_types]
        left = pack(demand, free)
        totals = [dict(n["total"]) for n in load["nodes"]]
        totals += [dict(cfg.node_types[t].resources) for _, t in launching
                   if t in cfg.node_types]
        left += pack(requested, totals)
        # 2) node types to launch for the leftovers (+ min_workers)
        count = {t: 0 for t in cfg.node_types}
        for t in workers.values():
            if t in count:
                count[t] += 1
        plan = {t: 0 for t in cfg.node_types}
        for t, nt in cfg.node_types.items():
            plan[t] = max(0, nt.min_workers - count[t])
        new_bins = []  # (type, remaining capacity) of nodes planned this round
        for t, n in plan.items():
            new_bins.extend((t, dict(cfg.node_types[t].resources)) for _ in range(n))
        for r in sorted(left, key=_size, reverse=True):
            for _, cap in new_bins:
                if _fits(cap, r):
                    _take(cap, r)
                    break
            else:
                choices = [(sum(nt.resources.values()), t) for t, nt in cfg.node_types.items()
                           if _fits(nt.resources, r) and
                           count[t] + plan[t] < nt.max_workers]
                if not choices:
                    continue  # infeasible for every node type (the raylet warns the user)
                _, t = min(choices)
                plan[t] += 1
                cap = dict(cfg.node_types[t].resources)
                _take(cap, r)
                new_bins.append((t, cap))
        # global cap and upscaling speed (at least 5 nodes per round, like the reference)
        room = max(0, cfg.max_workers - len(workers))
        speed = max(5, int(cfg.upscaling_speed * max(1, len(workers))))
        budget = min(room, speed)
        launched = []
        for t, n in plan.items():
            n = min(n, budget)
            if n <= 0:
                continue
            budget -= n
            nt = cfg.node_types[t]
            ids = self.provider.create_node(dict(nt.node_config, resources=nt.resources),
                                            {TAG_NODE_KIND: "worker", TAG_USER_NODE_TYPE: t}, n)
            now = time.time()
            for pid in ids:
                self.launched_at[pid] = now
                self.events.append((now, "launch", t, pid))
            launched.extend(ids)
        # 3) idle scale-down (never below min_workers, never with demand left unplaced)
        terminated = []
        if not left:
            alive = dict(count)
            for pid, t in workers.items():
                rn = joined.get(self.provider.ray_node_id(pid))
                if rn is None or rn["idle_s"] < cfg.idle_timeout_s:
                    continue
                if t in cfg.node_types and alive[t] <= cfg.node_types[t].min_workers:
                    continue
                self.provider.terminate_node(pid)
                alive[t] = alive.get(t, 1) - 1
                self.events.append((time.time(), "terminate", t, pid))
                terminated.append(pid)
        return {"launched": launched, "terminated": terminated, "unplaced": left}


class Monitor:
    """Runs ``StandardAutoscaler.update`` every ``update_interval_s`` on a thread
    (reference: autoscaler/_private/monitor.py)."""

    def __init__(self, autoscaler: StandardAutoscaler):
        self.autoscaler = autoscaler
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._run, name="ray_amd-autoscaler", daemon=True)
        self.errors = 0

    def start(self):
        self.thread.start()
        return self

    def _run(self):
        while not self._stop.wait(self.autoscaler.config.update_interval_s):
            try:
                self.autoscaler.update()
            except Exception as e:  # noqa: BLE001
                self.errors += 1
                print(f"[ray_amd] autoscaler update failed: {e!r}", file=sys.stderr,
                      flush=True)

    def stop(self):
        self._stop.set()
        self.thread.join(timeout=10)
