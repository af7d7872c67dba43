"""Distributed FIFO queue backed by an async actor (reference: python/ray/util/queue.py)."""

from __future__ import annotations

import asyncio
import queue as _q

import ray_amd as ray


class Empty(_q.Empty):
    pass


class Full(_q.Full):
    pass


class _QueueActor:
    def __init__(self, maxsize):
        self.maxsize = maxsize
        self.queue = asyncio.Queue(maxsize)

    def qsize(self):
        return self.queue.qsize()

    def empty(self):
        return self.queue.empty()

    def full(self):
        return self.queue.full()

    async def put(self, item, timeout=None):
        try:
            await asyncio.wait_for(self.queue.put(item), timeout)
        except asyncio.TimeoutError:
            raise Full

    async def put_batch(self, items, timeout=None):
        for item in items:
            try:
                await asyncio.wait_for(self.queue.put(item), timeout)
            except asyncio.TimeoutError:
                raise Full

    async def get(self, timeout=None):
        try:
            return await asyncio.wait_for(self.queue.get(), timeout)
        except asyncio.TimeoutError:
            raise Empty

    def put_nowait(self, item):
        self.queue.put_nowait(item)

    def put_nowait_batch(self, items):
        if self.maxsize > 0 and len(items) + self.qsize() > self.maxsize:
            raise Full(f"Cannot add {len(items)} items to queue of size {self.qsize()} and "
                       f"maxsize {self.maxsize}.")
        for item in items:
            self.queue.put_nowait(item)

    def get_nowait(self):
        return self.queue.get_nowait()

    def get_nowait_batch(self, num_items):
        if num_items > self.qsize():
            raise Empty(f"Cannot get {num_items} items from queue of size {self.qsize()}.")
        return [self.queue.get_nowait() for _ in range(num_items)]


class Queue:
    def __init__(self, maxsize: int = 0, actor_options: dict | None = None):
        self.maxsize = maxsize
        self.actor = ray.remote(_QueueActor).options(**(actor_options or {})).remote(maxsize)

    def __len__(self):
        return self.size()

    def size(self):
        return ray.get(self.actor.qsize.remote())

    def qsize(self):
        return self.size()

    def empty(self):
        return ray.get(self.actor.empty.remote())

    def full(self):
        return ray.get(self.actor.full.remote())

    def put(self, item, block=True, timeout=None):
        if not block:
            try:
                ray.get(self.actor.put_nowait.remote(item))
            except asyncio.QueueFull:
                raise Full
        else:
            if timeout is not None and timeout < 0:
                raise ValueError("'timeout' must be a non-negative number")
            ray.get(self.actor.put.remote(item, timeout))

    async def put_async(self, item, block=True, timeout=None):
        if not block:
            try:
                await self.actor.put_nowait.remote(item)
            except asyncio.QueueFull:
                raise Full
        else:
            await self.actor.put.remote(item, timeout)

    def get(self, block=True, timeout=None):
        if not block:
            try:
                return ray.get(self.actor.get_nowait.remote())
            except asyncio.QueueEmpty:
                raise Empty
        if timeout is not None and timeout < 0:
            raise ValueError("'timeout' must be a non-negative number")
        return ray.get(self.actor.get.remote(timeout))

    async def get_async(self, block=True, timeout=None):
        if not block:
            try:
                return await self.actor.get_nowait.remote()
            except asyncio.QueueEmpty:
                raise Empty
        return await self.actor.get.remote(timeout)

    def put_nowait(self, item):
        return self.put(item, block=False)

    def put_nowait_batch(self, items):
        if not isinstance(items, list):
            raise TypeError("Argument 'items' must be a list")
        ray.get(self.actor.put_nowait_batch.remote(items))

    def get_nowait(self):
        return self.get(block=False)

    def get_nowait_batch(self, num_items):
        if not isinstance(num_items, int) or num_items < 0:
            raise ValueError("'num_items' must be a nonnegative integer")
        return ray.get(self.actor.get_nowait_batch.remote(num_items))

    def shutdown(self, force=False, grace_period_s=5):
        if self.actor:
            ray.kill(self.actor)
        self.actor = None
