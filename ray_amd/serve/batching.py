"""@serve.batch dynamic request batching (reference: python/ray/serve/batching.py).

Concurrent calls to the decorated async method are queued; a background task
flushes a batch when ``max_batch_size`` requests are waiting or
``batch_wait_timeout_s`` has elapsed since the first one, calls the method once
with a list, and scatters the returned list back to the callers."""

from __future__ import annotations

import asyncio
import functools


class _Batcher:
    def __init__(self, fn, max_batch_size, timeout_s):
        self.fn = fn
        self.max = max_batch_size
        self.timeout = timeout_s
        self.queue = None
        self.task = None

    def _ensure(self):
        if self.queue is None:
            self.queue = asyncio.Queue()
            self.task = asyncio.get_running_loop().create_task(self._loop())

    async def _loop(self):
        while True:
            first = await self.queue.get()
            batch = [first]
            deadline = asyncio.get_running_loop().time() + self.timeout
            while len(batch) < self.max:
                rem = deadline - asyncio.get_running_loop().time()
                if rem <= 0:
                    break
                try:
                    batch.append(await asyncio.wait_for(self.queue.get(), rem))
                except asyncio.TimeoutError:
                    break
            selves = batch[0][0]
            args = [b[1] for b in batch]
            futs = [b[2] for b in batch]
            try:
                if selves is not None:
                    out = self.fn(selves, args)
                else:
                    out = self.fn(args)
                if asyncio.iscoroutine(out):
                    out = await out
                out = list(out)
                if len(out) != len(futs):
                    raise ValueError(f"batched function returned {len(out)} results for "
                                     f"{len(futs)} inputs")
                for f, o in zip(futs, out):
                    if not f.done():
                        f.set_result(o)
            except Exception as e:  # noqa: BLE001
                for f in futs:
                    if not f.done():
                        f.set_exception(e)

    async def submit(self, self_obj, arg):
        self._ensure()
        fut = asyncio.get_running_loop().create_future()
        await self.queue.put((self_obj, arg, fut))
        return await fut


def batch(_fn=None, *, max_batch_size: int = 10, batch_wait_timeout_s: float = 0.01):
    def deco(fn):
        batchers = {}

        @functools.wraps(fn)
        async def wrapper(*args):
            if len(args) == 2:
                self_obj, arg = args
            else:
                self_obj, arg = None, args[0]
            key = id(self_obj)
            b = batchers.get(key)
            if b is None:
                b = batchers[key] = _Batcher(fn, max_batch_size, batch_wait_timeout_s)
            return await b.submit(self_obj, arg)

        wrapper._is_serve_batch = True
        return wrapper

    if _fn is not None and callable(_fn):
        return deco(_fn)
    return deco
