"""@serve.batch dynamic request batching (reference: python/ray/serve/batching.py).

Concurrent calls to the decorated async method are queued; a background task
flushes a batch when ``max_batch_size`` requests are waiting or
``batch_wait_timeout_s`` has elapsed since the first one (requests already queued are
always taken, so a timeout of 0 still batches a burst), calls the method once with a
list, and scatters the returned list back to the callers.

An ``async def`` generator handler streams: each step it yields one list with an item
per request, and every caller iterates its own stream of items. ``set_max_batch_size``
/ ``set_batch_wait_timeout_s`` on the decorated method retune it at runtime (e.g. from
``reconfigure``)."""

from __future__ import annotations

import asyncio
import functools
import inspect

_END = object()


class _Batcher:
    def __init__(self, fn, params):
        self.fn = fn
        self.params = params  # shared, live-updated {"max": n, "timeout": s}
        self.stream = inspect.isasyncgenfunction(fn)
        self.queue = None
        self.task = None

    def _ensure(self):
        if self.queue is None:
            self.queue = asyncio.Queue()
            self.task = asyncio.get_running_loop().create_task(self._loop())

    async def _collect(self):
        first = await self.queue.get()
        batch = [first]
        loop = asyncio.get_running_loop()
        deadline = loop.time() + self.params["timeout"]
        while len(batch) < self.params["max"]:
            try:  # whatever is already queued joins without waiting
                batch.append(self.queue.get_nowait())
                continue
            except asyncio.QueueEmpty:
                pass
            rem = deadline - loop.time()
            if rem <= 0:
                break
            try:
                batch.append(await asyncio.wait_for(self.queue.get(), rem))
            except asyncio.TimeoutError:
                break
        return batch

    def _call(self, selves, args):
        return self.fn(selves, args) if selves is not None else self.fn(args)

    async def _loop(self):
        while True:
            batch = await self._collect()
            selves = batch[0][0]
            args = [b[1] for b in batch]
            sinks = [b[2] for b in batch]
            try:
                if self.stream:
                    async for out in self._call(selves, args):
                        out = list(out)
                        if len(out) != len(sinks):
                            raise ValueError(f"batched generator yielded {len(out)} results "
                                             f"for {len(sinks)} inputs")
                        for q, o in zip(sinks, out):
                            q.put_nowait(o)
                    for q in sinks:
                        q.put_nowait(_END)
                    continue
                out = self._call(selves, args)
                if asyncio.iscoroutine(out):
                    out = await out
                out = list(out)
                if len(out) != len(sinks):
                    raise ValueError(f"batched function returned {len(out)} results for "
                                     f"{len(sinks)} inputs")
                for f, o in zip(sinks, out):
                    if not f.done():
                        f.set_result(o)
            except Exception as e:  # noqa: BLE001
                for s in sinks:
                    if self.stream:
                        s.put_nowait(_Raise(e))
                    elif not s.done():
                        s.set_exception(e)

    async def submit(self, self_obj, arg):
        self._ensure()
        fut = asyncio.get_running_loop().create_future()
        await self.queue.put((self_obj, arg, fut))
        return await fut

    async def submit_stream(self, self_obj, arg):
        self._ensure()
        q = asyncio.Queue()
        await self.queue.put((self_obj, arg, q))
        while True:
            item = await q.get()
            if item is _END:
                return
            if isinstance(item, _Raise):
                raise item.exc
            yield item


class _Raise:
    __slots__ = ("exc",)

    def __init__(self, exc):
        self.exc = exc


def _check(max_batch_size, batch_wait_timeout_s):
    if not isinstance(max_batch_size, int) or max_batch_size < 1:
        raise ValueError("max_batch_size must be an integer >= 1")
    if not isinstance(batch_wait_timeout_s, (int, float)) or batch_wait_timeout_s < 0:
        raise TypeError("batch_wait_timeout_s must be a float >= 0")


def batch(_fn=None, *, max_batch_size: int = 10, batch_wait_timeout_s: float = 0.0):
    _check(max_batch_size, batch_wait_timeout_s)

    def deco(fn):
        if not (inspect.iscoroutinefunction(fn) or inspect.isasyncgenfunction(fn)):
            raise TypeError("Functions decorated with @serve.batch must be 'async def'")
        params = {"max": max_batch_size, "timeout": float(batch_wait_timeout_s)}
        batchers = {}

        def batcher(args):
            if len(args) == 2:
                self_obj, arg = args
            elif len(args) == 1:
                self_obj, arg = None, args[0]
            else:
                raise TypeError("@serve.batch methods take exactly one argument per call")
            key = id(self_obj)
            b = batchers.get(key)
            if b is None:
                b = batchers[key] = _Batcher(fn, params)
            return b, self_obj, arg

        if inspect.isasyncgenfunction(fn):
            @functools.wraps(fn)
            async def wrapper(*args):
                b, self_obj, arg = batcher(args)
                async for item in b.submit_stream(self_obj, arg):
                    yield item
        else:
            @functools.wraps(fn)
            async def wrapper(*args):
                b, self_obj, arg = batcher(args)
                return await b.submit(self_obj, arg)

        def set_max_batch_size(n: int) -> None:
            _check(n, params["timeout"])
            params["max"] = n

        def set_batch_wait_timeout_s(t: float) -> None:
            _check(params["max"], t)
            params["timeout"] = float(t)

        wrapper._is_serve_batch = True
        wrapper.set_max_batch_size = set_max_batch_size
        wrapper.set_batch_wait_timeout_s = set_batch_wait_timeout_s
        wrapper._get_max_batch_size = lambda: params["max"]
        wrapper._get_batch_wait_timeout_s = lambda: params["timeout"]
        return wrapper

    if _fn is not None and callable(_fn):
        return deco(_fn)
    return deco
