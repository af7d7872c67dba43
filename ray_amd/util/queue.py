"""Distributed FIFO queue served by one async actor.

API contract (reference: python/ray/util/queue.py — ``Queue(maxsize, actor_options)``
with ``put/get`` (block, timeout), ``*_nowait``, ``*_nowait_batch``, ``put_async``,
``get_async``, ``qsize/size/empty/full``, ``shutdown``, and the ``Empty``/``Full``
exceptions, which subclass the stdlib ``queue`` ones).

Design: the actor keeps a ``collections.deque`` and ONE ``asyncio.Condition``; every
operation is a single actor call that moves a whole batch at once (``push_items`` /
``pop_items`` take lists), blocking callers park on the condition with their own
deadline, so a blocked ``get`` costs no polling and does not hold up other callers
(the actor is async: one event loop, many waiting coroutines).
"""

from __future__ import annotations

import asyncio
import collections
import queue as _stdlib_queue
import time

import ray_amd as ray


class Empty(_stdlib_queue.Empty):
    pass


class Full(_stdlib_queue.Full):
    pass


class _QueueActor:
    def __init__(self, maxsize: int):
        self.cap = maxsize if maxsize and maxsize > 0 else None
        self.items: collections.deque = collections.deque()
        self.cond = None  # created lazily inside the actor's event loop

    def _cv(self):
        if self.cond is None:
            self.cond = asyncio.Condition()
        return self.cond

    def size(self):
        return len(self.items)

    def room(self):
        return None if self.cap is None else self.cap - len(self.items)

    async def push_items(self, batch: list, block: bool, timeout):
        cv = self._cv()
        n = len(batch)
        if self.cap is not None and n > self.cap:
            raise Full(f"cannot put {n} items into a queue of maxsize {self.cap}")
        deadline = None if timeout is None else time.monotonic() + timeout
        async with cv:
            while self.cap is not None and len(self.items) + n > self.cap:
                if not block:
                    raise Full(f"queue full ({len(self.items)}/{self.cap}); cannot add {n}")
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    raise Full("timed out waiting for free space")
                try:
                    await asyncio.wait_for(cv.wait(), left)
                except asyncio.TimeoutError:
                    raise Full("timed out waiting for free space") from None
            self.items.extend(batch)
            cv.notify_all()

    async def pop_items(self, n: int, block: bool, timeout):
        cv = self._cv()
        deadline = None if timeout is None else time.monotonic() + timeout
        async with cv:
            while len(self.items) < n:
                if not block:
                    raise Empty(f"queue holds {len(self.items)} items; {n} requested")
                left = None if deadline is None else deadline - time.monotonic()
                if left is not None and left <= 0:
                    raise Empty("timed out waiting for an item")
                try:
                    await asyncio.wait_for(cv.wait(), left)
                except asyncio.TimeoutError:
                    raise Empty("timed out waiting for an item") from None
            out = [self.items.popleft() for _ in range(n)]
            cv.notify_all()
            return out


def _check_timeout(timeout):
    if timeout is not None and timeout < 0:
        raise ValueError("'timeout' must be a non-negative number")


class Queue:
    def __init__(self, maxsize: int = 0, actor_options: dict | None = None):
        self.maxsize = maxsize
        opts = dict(actor_options or {})
        opts.setdefault("max_concurrency", 1000)  # many parked put/get coroutines
        self.actor = ray.remote(_QueueActor).options(**opts).remote(maxsize)

    # -------------------------------------------------------------- introspection
    def __len__(self):
        return self.size()

    def size(self) -> int:
        return ray.get(self.actor.size.remote())

    qsize = size

    def empty(self) -> bool:
        return self.size() == 0

    def full(self) -> bool:
        if not self.maxsize or self.maxsize <= 0:
            return False
        return ray.get(self.actor.room.remote()) <= 0

    # -------------------------------------------------------------- put
    def put(self, item, block: bool = True, timeout=None) -> None:
        _check_timeout(timeout)
        ray.get(self.actor.push_items.remote([item], block, timeout))

    async def put_async(self, item, block: bool = True, timeout=None) -> None:
        _check_timeout(timeout)
        await self.actor.push_items.remote([item], block, timeout)

    def put_nowait(self, item) -> None:
        self.put(item, block=False)

    def put_nowait_batch(self, items) -> None:
        if not isinstance(items, list):
            raise TypeError("Argument 'items' must be a list")
        ray.get(self.actor.push_items.remote(list(items), False, None))

    # -------------------------------------------------------------- get
    def get(self, block: bool = True, timeout=None):
        _check_timeout(timeout)
        return ray.get(self.actor.pop_items.remote(1, block, timeout))[0]

    async def get_async(self, block: bool = True, timeout=None):
        _check_timeout(timeout)
        return (await self.actor.pop_items.remote(1, block, timeout))[0]

    def get_nowait(self):
        return self.get(block=False)

    def get_nowait_batch(self, num_items: int) -> list:
        if not isinstance(num_items, int) or num_items < 0:
            raise ValueError("'num_items' must be a nonnegative integer")
        return ray.get(self.actor.pop_items.remote(num_items, False, None))

    def shutdown(self, force: bool = False, grace_period_s: int = 5) -> None:
        if self.actor is not None:
            ray.kill(self.actor)
        self.actor = None
