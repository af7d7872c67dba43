"""ActorPool: schedule a stream of calls over a fixed set of actors.

API contract (reference: python/ray/util/actor_pool.py — ``map``, ``map_unordered``,
``submit``, ``has_next``, ``get_next``, ``get_next_unordered``, ``has_free``,
``pop_idle``, ``push``).

Design: every submission is a ``_Job`` that moves through
``queued -> running -> ready -> consumed``. Queued jobs wait in a backlog until an
actor is free; a running job's actor is released the moment its result is known to be
ready (``ready``), so the backlog keeps draining while the caller has not consumed the
value yet. One deque keeps the unconsumed jobs in submission order, so ordered and
unordered retrieval can be mixed freely: ``get_next`` returns the oldest unconsumed
result, ``get_next_unordered`` whichever is ready first.
"""

from __future__ import annotations

import collections
from typing import Any, Callable, Iterable

import ray_amd as ray

_QUEUED, _RUNNING, _READY, _CONSUMED = range(4)


class _Job:
    __slots__ = ("fn", "value", "ref", "actor", "state")

    def __init__(self, fn: Callable, value: Any):
        self.fn, self.value = fn, value
        self.ref = self.actor = None
        self.state = _QUEUED


class ActorPool:
    def __init__(self, actors: list):
        self._free: collections.deque = collections.deque(actors)
        self._backlog: collections.deque[_Job] = collections.deque()
        self._running: dict = {}  # ObjectRef -> _Job
        self._order: collections.deque[_Job] = collections.deque()  # unconsumed jobs

    # -------------------------------------------------------------- scheduling
    def _dispatch(self):
        while self._free and self._backlog:
            job = self._backlog.popleft()
            job.actor = self._free.popleft()
            job.ref = job.fn(job.actor, job.value)
            job.state = _RUNNING
            self._running[job.ref] = job

    def _mark_ready(self, job: _Job):
        del self._running[job.ref]
        job.state = _READY
        self._free.append(job.actor)
        job.actor = None
        self._dispatch()

    def _consume(self, job: _Job):
        job.state = _CONSUMED
        while self._order and self._order[0].state == _CONSUMED:
            self._order.popleft()
        return ray.get(job.ref)

    def _wait(self, refs, timeout, ignore_if_timedout):
        ready, _ = ray.wait(refs, num_returns=1, timeout=timeout)
        if ready:
            return ready[0]
        if ignore_if_timedout:
            return None
        raise TimeoutError("Timed out waiting for result")

    def submit(self, fn: Callable, value) -> None:
        """Schedule ``fn(actor, value)`` (which must return an ObjectRef) on a free actor,
        or queue it until one frees up."""
        job = _Job(fn, value)
        self._backlog.append(job)
        self._order.append(job)
        self._dispatch()

    # -------------------------------------------------------------- retrieval
    def has_next(self) -> bool:
        return bool(self._order)

    def get_next(self, timeout=None, ignore_if_timedout=False):
        """Result of the oldest unconsumed submission (blocking)."""
        if not self._order:
            raise StopIteration("No more results to get")
        job = self._order[0]
        while job.state == _QUEUED:  # free an actor for it: wait for any running job
            ref = self._wait(list(self._running), timeout, ignore_if_timedout)
            if ref is None:
                return None
            self._mark_ready(self._running[ref])
        if job.state == _RUNNING:
            if self._wait([job.ref], timeout, ignore_if_timedout) is None:
                return None
            self._mark_ready(job)
        return self._consume(job)

    def get_next_unordered(self, timeout=None, ignore_if_timedout=False):
        """Result of whichever unconsumed submission is ready first."""
        if not self._order:
            raise StopIteration("No more results to get")
        for job in self._order:  # already known ready (released early by get_next)
            if job.state == _READY:
                return self._consume(job)
        if not self._running:
            raise RuntimeError("ActorPool has queued work but no actors")
        ref = self._wait(list(self._running), timeout, ignore_if_timedout)
        if ref is None:
            return None
        job = self._running[ref]
        self._mark_ready(job)
        return self._consume(job)

    def map(self, fn: Callable, values: Iterable):
        """Apply ``fn(actor, v)`` to every value (submitted now); results in input order."""
        for v in values:
            self.submit(fn, v)
        return self._drain(self.get_next)

    def map_unordered(self, fn: Callable, values: Iterable):
        """Like ``map`` but yields results as they complete."""
        for v in values:
            self.submit(fn, v)
        return self._drain(self.get_next_unordered)

    def _drain(self, get):
        while self.has_next():
            yield get()

    # -------------------------------------------------------------- membership
    def has_free(self) -> bool:
        return bool(self._free) and not self._backlog

    def pop_idle(self):
        """Remove and return an idle actor (None if none is idle)."""
        return self._free.popleft() if self.has_free() else None

    def push(self, actor) -> None:
        """Add an actor to the pool (it immediately takes queued work)."""
        busy = [j.actor for j in self._running.values()]
        if actor in self._free or actor in busy:
            raise ValueError("Actor already belongs to current ActorPool")
        self._free.append(actor)
        self._dispatch()
