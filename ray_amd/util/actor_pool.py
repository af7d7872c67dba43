"""ActorPool (reference: python/ray/util/actor_pool.py)."""

from __future__ import annotations

import ray_amd as ray


class ActorPool:
    def __init__(self, actors: list):
        self._idle_actors = list(actors)
        self._future_to_actor = {}
        self._index_to_future = {}
        self._next_task_index = 0
        self._next_return_index = 0
        self._pending_submits = []

    def map(self, fn, values):
        while self.has_next():
            try:
                self.get_next_unordered(timeout=0)
            except TimeoutError:
                break
        for v in values:
            self.submit(fn, v)

        def gen():
            while self.has_next():
                yield self.get_next()

        return gen()

    def map_unordered(self, fn, values):
        for v in values:
            self.submit(fn, v)

        def gen():
            while self.has_next():
                yield self.get_next_unordered()

        return gen()

    def submit(self, fn, value):
        if self._idle_actors:
            actor = self._idle_actors.pop()
            future = fn(actor, value)
            key = future
            self._future_to_actor[key] = (self._next_task_index, actor)
            self._index_to_future[self._next_task_index] = future
            self._next_task_index += 1
        else:
            self._pending_submits.append((fn, value))

    def has_next(self):
        return bool(self._future_to_actor)

    def get_next(self, timeout=None, ignore_if_timedout=False):
        if not self.has_next():
            raise StopIteration("No more results to get")
        if self._next_return_index >= self._next_task_index:
            raise ValueError("It is not allowed to call get_next() after get_next_unordered().")
        future = self._index_to_future[self._next_return_index]
        if timeout is not None:
            res, _ = ray.wait([future], timeout=timeout)
            if not res:
                if not ignore_if_timedout:
                    raise TimeoutError("Timed out waiting for result")
                return None
        del self._index_to_future[self._next_return_index]
        self._next_return_index += 1
        i, a = self._future_to_actor.pop(future)
        self._return_actor(a)
        return ray.get(future)

    def get_next_unordered(self, timeout=None, ignore_if_timedout=False):
        if not self.has_next():
            raise StopIteration("No more results to get")
        res, _ = ray.wait(list(self._future_to_actor), num_returns=1, timeout=timeout)
        if not res:
            if ignore_if_timedout:
                return None
            raise TimeoutError("Timed out waiting for result")
        future = res[0]
        i, a = self._future_to_actor.pop(future)
        self._return_actor(a)
        del self._index_to_future[i]
        self._next_return_index = max(self._next_return_index, i + 1)
        return ray.get(future)

    def _return_actor(self, actor):
        self._idle_actors.append(actor)
        if self._pending_submits:
            self.submit(*self._pending_submits.pop(0))

    def has_free(self):
        return bool(self._idle_actors) and not self._pending_submits

    def pop_idle(self):
        return self._idle_actors.pop() if self.has_free() else None

    def push(self, actor):
        busy = [a for _, a in self._future_to_actor.values()]
        if actor in self._idle_actors or actor in busy:
            raise ValueError("Actor already belongs to current ActorPool")
        self._return_actor(actor)
