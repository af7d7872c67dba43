"""FaultTolerantActorManager (reference: rllib/utils/actor_manager.py:193).

Holds a group of actors by id, runs calls on every healthy one and reports per-actor
success or failure instead of raising on the first dead actor; ``probe_unhealthy_actors``
pings the ones marked unhealthy (and, with ``restore``, recreates dead ones through the
caller's factory). Algorithm uses it for its EnvRunners (AlgorithmConfig.fault_tolerance).
"""

from __future__ import annotations

import time

import ray_amd as ray
from ray_amd.exceptions import GetTimeoutError, RayActorError


class CallResult:
    __slots__ = ("actor_id", "ok", "value")

    def __init__(self, actor_id, ok, value):
        self.actor_id, self.ok, self.value = actor_id, ok, value

    def get(self):
        if not self.ok:
            raise self.value
        return self.value


def _is_actor_failure(e) -> bool:
    return isinstance(e, (RayActorError, GetTimeoutError))


class FaultTolerantActorManager:
    def __init__(self, actors=None, *, max_remote_requests_in_flight_per_actor: int = 2,
                 init_id: int = 1, restore_fn=None):
        self._actors = {}
        self._healthy = {}
        self._restore_fn = restore_fn  # actor_id -> new actor handle (or None)
        self.num_restarts = 0
        self.num_failures = 0
        self._next_id = init_id
        self.max_in_flight = max_remote_requests_in_flight_per_actor
        self._inflight = {}  # ref -> actor_id
        for a in actors or ():
            self.add_actors([a])

    # ---------------------------------------------------------------- membership
    def add_actors(self, actors):
        ids = []
        for a in actors:
            i = self._next_id
            self._next_id += 1
            self._actors[i] = a
            self._healthy[i] = True
            ids.append(i)
        return ids

    def remove_actor(self, actor_id):
        self._healthy.pop(actor_id, None)
        return self._actors.pop(actor_id, None)

    def actor_ids(self):
        return list(self._actors)

    def healthy_actor_ids(self):
        return [i for i, h in self._healthy.items() if h]

    def num_actors(self):
        return len(self._actors)

    def num_healthy_actors(self):
        return len(self.healthy_actor_ids())

    def actors(self, healthy_only=True):
        ids = self.healthy_actor_ids() if healthy_only else self.actor_ids()
        return [self._actors[i] for i in ids]

    def get(self, actor_id):
        return self._actors[actor_id]

    def set_actor_state(self, actor_id, healthy: bool):
        if actor_id in self._actors:
            was = self._healthy.get(actor_id)
            self._healthy[actor_id] = healthy
            if was and not healthy:
                self.num_failures += 1

    # ---------------------------------------------------------------- calls
    def foreach_actor(self, fn, *, healthy_only=True, remote_actor_ids=None, timeout_s=None,
                      mark_healthy=False):
        """fn(actor) -> ObjectRef (or a method name + args via a lambda); returns a list of
        CallResult. Actors whose call fails with an actor error are marked unhealthy."""
        ids = remote_actor_ids if remote_actor_ids is not None else (
            self.healthy_actor_ids() if healthy_only else self.actor_ids())
        refs = []
        for i in ids:
            try:
                refs.append((i, fn(self._actors[i])))
            except Exception as e:  # noqa: BLE001  (submission to a dead actor)
                refs.append((i, e))
        out = []
        deadline = None if timeout_s is None else time.time() + timeout_s
        for i, ref in refs:
            if isinstance(ref, BaseException):
                self.set_actor_state(i, False)
                out.append(CallResult(i, False, ref))
                continue
            try:
                left = None if deadline is None else max(0.0, deadline - time.time())
                v = ray.get(ref, timeout=left)
                out.append(CallResult(i, True, v))
                if mark_healthy:
                    self.set_actor_state(i, True)
            except Exception as e:  # noqa: BLE001
                if _is_actor_failure(e):
                    self.set_actor_state(i, False)
                out.append(CallResult(i, False, e))
        return out

    def foreach_actor_async(self, fn, *, remote_actor_ids=None):
        """Submit fn(actor) on healthy actors with fewer than max_in_flight requests;
        returns the number submitted. Collect with fetch_ready_async_reqs."""
        per = {}
        for aid in self._inflight.values():
            per[aid] = per.get(aid, 0) + 1
        n = 0
        for i in (remote_actor_ids or self.healthy_actor_ids()):
            if per.get(i, 0) >= self.max_in_flight or not self._healthy.get(i):
                continue
            try:
                self._inflight[fn(self._actors[i])] = i
                n += 1
            except Exception:  # noqa: BLE001
                self.set_actor_state(i, False)
        return n

    def fetch_ready_async_reqs(self, *, timeout_seconds=0.0, return_obj_refs=False):
        if not self._inflight:
            return []
        ready, _ = ray.wait(list(self._inflight), num_returns=len(self._inflight),
                            timeout=timeout_seconds)
        out = []
        for ref in ready:
            i = self._inflight.pop(ref)
            if return_obj_refs:
                out.append(CallResult(i, True, ref))
                continue
            try:
                out.append(CallResult(i, True, ray.get(ref)))
            except Exception as e:  # noqa: BLE001
                if _is_actor_failure(e):
                    self.set_actor_state(i, False)
                out.append(CallResult(i, False, e))
        return out

    def num_outstanding_async_reqs(self):
        return len(self._inflight)

    # ---------------------------------------------------------------- recovery
    def probe_unhealthy_actors(self, timeout_seconds: float = 30.0, restore=True,
                               mark_healthy=True):
        """Ping every actor marked unhealthy; a live one is marked healthy again, a dead
        one is recreated through ``restore_fn`` (when given). Returns the restored ids."""
        restored = []
        for i in [i for i, h in self._healthy.items() if not h]:
            alive = False
            try:
                ray.get(self._actors[i].ping.remote(), timeout=timeout_seconds)
                alive = True
            except Exception:  # noqa: BLE001
                alive = False
            if alive:
                if mark_healthy:
                    self._healthy[i] = True
                continue
            if restore and self._restore_fn is not None:
                try:
                    ray.kill(self._actors[i])
                except Exception:  # noqa: BLE001
                    pass
                new = self._restore_fn(i)
                if new is not None:
                    self._actors[i] = new
                    self._healthy[i] = True
                    self.num_restarts += 1
                    restored.append(i)
                    for ref in [r for r, a in self._inflight.items() if a == i]:
                        self._inflight.pop(ref, None)
        return restored

    def clear(self):
        for a in self._actors.values():
            try:
                ray.kill(a)
            except Exception:  # noqa: BLE001
                pass
        self._actors.clear()
        self._healthy.clear()
        self._inflight.clear()
