"""multiprocessing.Pool API on ray_amd actors (reference: python/ray/util/multiprocessing/pool.py)."""

from __future__ import annotations

import itertools
import os
import time

import ray_amd as ray


class _PoolActor:
    def __init__(self, initializer=None, initargs=None):
        if initializer:
            initializer(*(initargs or ()))

    def ping(self):
        return os.getpid()

    def run_batch(self, func, batch, star):
        out = []
        for args in batch:
            try:
                out.append((True, func(*args) if star else func(args)))
            except Exception as e:  # noqa: BLE001
                out.append((False, e))
        return out


class AsyncResult:
    def __init__(self, refs, single, callback=None, error_callback=None, flatten=True):
        self._refs = refs
        self._single = single
        self._callback = callback
        self._error_callback = error_callback
        self._value = None
        self._done = False

    def _fetch(self, timeout=None):
        if self._done:
            return
        ready, _ = ray.wait(self._refs, num_returns=len(self._refs), timeout=timeout)
        if len(ready) < len(self._refs):
            raise TimeoutError
        vals = []
        for batch in ray.get(self._refs):
            vals.extend(batch)
        self._done = True
        self._value = vals
        err = next((v for ok, v in vals if not ok), None)
        if err is not None:
            if self._error_callback:
                self._error_callback(err)
        elif self._callback:
            res = [v for _, v in vals]
            self._callback(res[0] if self._single else res)

    def get(self, timeout=None):
        self._fetch(timeout)
        for ok, v in self._value:
            if not ok:
                raise v
        res = [v for _, v in self._value]
        return res[0] if self._single else res

    def wait(self, timeout=None):
        try:
            self._fetch(timeout)
        except TimeoutError:
            pass

    def ready(self):
        if self._done:
            return True
        r, _ = ray.wait(self._refs, num_returns=len(self._refs), timeout=0)
        return len(r) == len(self._refs)

    def successful(self):
        if not self.ready():
            raise ValueError("result not ready")
        self._fetch()
        return all(ok for ok, _ in self._value)


class Pool:
    def __init__(self, processes: int | None = None, initializer=None, initargs=None,
                 maxtasksperchild=None, context=None, ray_address=None, ray_remote_args=None):
        if not ray.is_initialized():
            ray.init(address=ray_address)
        if processes is None:
            processes = int(ray.cluster_resources().get("CPU", 1))
        if processes <= 0:
            raise ValueError("Processes in the pool must be >0.")
        cls = ray.remote(_PoolActor).options(**(ray_remote_args or {"num_cpus": 1}))
        self._actors = [cls.remote(initializer, initargs) for _ in range(processes)]
        ray.get([a.ping.remote() for a in self._actors])
        self._rr = itertools.cycle(range(processes))
        self._closed = False
        self._processes = processes

    def _check(self):
        if self._closed:
            raise ValueError("Pool not running")

    def _submit(self, func, iterable, chunksize, star):
        items = list(iterable)
        if chunksize is None:
            chunksize, extra = divmod(len(items), self._processes * 4)
            if extra:
                chunksize += 1
            chunksize = max(1, chunksize)
        refs = []
        for i in range(0, len(items), chunksize):
            a = self._actors[next(self._rr)]
            refs.append(a.run_batch.remote(func, items[i:i + chunksize], star))
        return refs

    def apply(self, func, args=(), kwds=None):
        return self.apply_async(func, args, kwds).get()

    def apply_async(self, func, args=(), kwds=None, callback=None, error_callback=None):
        self._check()
        kw = kwds or {}
        f = (lambda *a: func(*a, **kw)) if kw else func
        refs = self._submit(f, [tuple(args)], 1, True)
        return AsyncResult(refs, True, callback, error_callback)

    def map(self, func, iterable, chunksize=None):
        return self.map_async(func, iterable, chunksize).get()

    def map_async(self, func, iterable, chunksize=None, callback=None, error_callback=None):
        self._check()
        return AsyncResult(self._submit(func, iterable, chunksize, False), False, callback,
                           error_callback)

    def starmap(self, func, iterable, chunksize=None):
        self._check()
        return AsyncResult(self._submit(func, iterable, chunksize, True), False).get()

    def starmap_async(self, func, iterable, chunksize=None, callback=None, error_callback=None):
        self._check()
        return AsyncResult(self._submit(func, iterable, chunksize, True), False, callback,
                           error_callback)

    def imap(self, func, iterable, chunksize=1):
        self._check()
        refs = self._submit(func, iterable, chunksize, False)
        for r in refs:
            for ok, v in ray.get(r):
                if not ok:
                    raise v
                yield v

    def imap_unordered(self, func, iterable, chunksize=1):
        self._check()
        refs = self._submit(func, iterable, chunksize, False)
        pending = list(refs)
        while pending:
            ready, pending = ray.wait(pending, num_returns=1)
            for ok, v in ray.get(ready[0]):
                if not ok:
                    raise v
                yield v

    def close(self):
        self._closed = True

    def terminate(self):
        self._closed = True
        for a in self._actors:
            ray.kill(a)
        self._actors = []

    def join(self):
        if not self._closed:
            raise ValueError("Pool is still running")
        time.sleep(0)

    def __enter__(self):
        self._check()
        return self

    def __exit__(self, *a):
        self.terminate()
